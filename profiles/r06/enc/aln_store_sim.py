#!/usr/bin/env python3
"""Host model of the aligned payload stores of the chunk-CRC tile encode (round 6,
tiles_group_kernel<…, ALN = true>): replays every store a work item of 2 chunks makes — lane
(chunk q, slot i = 8·ti + g, row r) per step — with the tail box and head box, and checks that
every payload word of every chunk is written exactly once with its value, that nothing outside
the chunk's payload is written, and which stores are whole 32-B sectors.  Run before the kernel
touches a GPU (a wrong address there is a memory fault)."""
import itertools

ROWS, TG = 32, 4


def simulate(units, m, d0_words):
    """One chunk whose payload starts at word address d0_words (m = d0_words mod 8).
    Returns {word address: value} of all stores and the list of store ops (addr, nwords)."""
    run_words = 32 * TG          # 128 words per row per step
    row_words = 32 * units       # payload row pitch (words)
    mem, ops = {}, []
    tail = {}                    # tail box[r][b]
    head = {}                    # head box[r][b]

    def R(r, s, w):              # value of run word w of row r, step s
        return ("v", r, s * run_words + w)

    def put(addr, val):
        assert addr not in mem, f"double write at {addr}"
        mem[addr] = val

    steps = units // TG
    for s in range(steps):
        first, last = s == 0, s == steps - 1
        for r in range(ROWS):
            rs = d0_words + r * row_words + s * run_words
            for i in range(32):
                wa = rs - m + 4 * i
                words = [4 * i + j - m for j in range(4)]
                if m == 0 or i >= 2:
                    vals = [R(r, s, w) for w in words]
                    for j in range(4):
                        put(wa + j, vals[j])
                    ops.append((wa, 4))
                    continue
                # slots 0, 1 of a misaligned run
                if first:
                    if r > 0:
                        for w in words:
                            if w >= 0:
                                head[(r, w)] = R(r, 0, w)
                    else:
                        for j, w in enumerate(words):
                            if w >= 0:
                                put(wa + j, R(r, 0, w))
                                ops.append((wa + j, 1))
                else:
                    vals = [tail[(r, w + m)] if w < 0 else R(r, s, w) for w in words]
                    for j in range(4):
                        put(wa + j, vals[j])
                    ops.append((wa, 4))
                if not last:  # this step's tail for the next step (own box words only)
                    for b in range(4 * i, 4 * i + 4):
                        if b < m:
                            tail[(r, b)] = R(r, s, run_words - m + b)
                else:          # the sector at the row's end: tail + the next row's head
                    end = rs + run_words
                    for j in range(4):
                        b = 4 * i + j
                        if b < m:
                            put(end - m + b, R(r, s, run_words - m + b))
                            ops.append((end - m + b, 1) if r == ROWS - 1 else None)
                        elif r < ROWS - 1:
                            put(end - m + b, head[(r + 1, b - m)])
                    if r < ROWS - 1:
                        ops.append((end - m + 4 * i, 4))
    return mem, [o for o in ops if o]


def check(units, m):
    d0 = 8 * 1000 + m
    mem, ops = simulate(units, m, d0)
    row_words = 32 * units
    want = {}
    for r in range(ROWS):
        for k in range(row_words):
            want[d0 + r * row_words + k] = ("v", r, k)
    assert set(mem) == set(want), (units, m, len(mem), len(want),
                                   sorted(set(mem) ^ set(want))[:8])
    for a, v in want.items():
        assert mem[a] == v, (a, mem[a], v)
    full = sum(1 for a, n in ops if n == 4 and (a % 4 == 0))
    part = sum(1 for a, n in ops if n == 1)
    return full, part


if __name__ == "__main__":
    for units, m in itertools.product((8, 12, 16, 32), range(8)):
        full, part = check(units, m)
        print(f"units {units:2d} m {m}: ok, {full} 16-B stores, {part} single-word stores")
    print("all layouts: every payload word written once, nothing outside the payload")
