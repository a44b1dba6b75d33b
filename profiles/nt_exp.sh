mkdir -p gpurun_out/s5
for cfg in c4crc c3crc c3nest; do
  for nt in 3 2; do
    ZH_NT=$nt timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline > gpurun_out/s5/${cfg}_nt$nt.json 2> gpurun_out/s5/${cfg}_nt$nt.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/s5/${cfg}_nt$nt.json'));print('$cfg nt$nt', d['value'], d['roofline']['kernel_ms'])"
  done
done
