"""Type check of the Java ↔ C boundary without a JDK: every `static native` method of
ZarrHip.java against the JNI function that implements it in zarrhip_jni.c.

There is no javac/javah here, so `javah`'s job is restated: each Java parameter
type maps to its JNI C type (JNI specification, "JNI Types and Data Structures": primitives to
jint/jlong/..., primitive arrays to j<prim>Array, String to jstring, any array of objects to
jobjectArray, other references to jobject), a static native method takes (JNIEnv*, jclass) first,
and the return type maps the same way.  The test compares arity, every parameter type and the
return type, so a jintArray/jlongArray swap or a dropped argument fails here instead of crashing
a JVM.  Reference surface the natives serve: v3.Array (/root/reference/src/main/java/dev/zarr/
zarrjava/v3/Array.java:28) and core.Array.read (core/Array.java:378)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "zarr-java_amd", "java", "src", "main", "java", "dev", "zarr",
                    "zarrjava", "hip", "ZarrHip.java")
JNI_C = os.path.join(ROOT, "zarr-java_amd", "java", "jni", "zarrhip_jni.c")
PREFIX = "Java_dev_zarr_zarrjava_hip_ZarrHip_"

PRIM = {"boolean": "jboolean", "byte": "jbyte", "char": "jchar", "short": "jshort",
        "int": "jint", "long": "jlong", "float": "jfloat", "double": "jdouble", "void": "void"}
REF = {"String": "jstring", "java.lang.String": "jstring", "Class": "jclass",
       "java.lang.Class": "jclass", "Throwable": "jthrowable", "java.lang.Throwable": "jthrowable"}


def jni_type(java_type):
    """The JNI C type of a Java parameter / return type (javah's mapping)."""
    t = java_type.replace(" ", "")
    dims = t.count("[]")
    base = t.replace("[]", "")
    if dims == 0:
        return PRIM.get(base) or REF.get(base) or "jobject"
    if dims == 1 and base in PRIM and base != "void":
        return PRIM[base] + "Array"
    return "jobjectArray"


def strip_comments(src, c_style=True):
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", " ", src)


def java_natives(src):
    """{name: (return JNI type, [parameter JNI types])} of every static native method."""
    out = {}
    pat = re.compile(r"static\s+native\s+([\w.\[\]\s]+?)\s+(\w+)\s*\(([^)]*)\)", re.S)
    for ret, name, params in pat.findall(strip_comments(src)):
        types = []
        for p in [x.strip() for x in params.split(",") if x.strip()]:
            p = re.sub(r"\bfinal\s+", "", p)
            m = re.match(r"(.+?)\s*(\w+)$", p, re.S)
            assert m, p
            types.append(jni_type(m.group(1)))
        assert name not in out, f"overloaded native {name}: JNI would need long names"
        out[name] = (jni_type(ret.strip()), types)
    return out


def c_natives(src):
    """{name: (return type, [parameter types after (JNIEnv*, jclass)])} of every JNI function."""
    out = {}
    pat = re.compile(r"JNIEXPORT\s+(\w+)\s+JNICALL\s+" + PREFIX + r"(\w+)\s*\(([^)]*)\)", re.S)
    for ret, name, params in pat.findall(strip_comments(src)):
        ps = [" ".join(x.split()) for x in params.split(",")]
        types = []
        for p in ps:
            m = re.match(r"(.+?)\s*\**\s*(\w+)$", p)
            assert m, p
            t = m.group(1).replace(" ", "")
            stars = p.count("*")
            types.append(t + "*" * stars if "*" not in t else t)
        assert types[:2] == ["JNIEnv*", "jclass"], (name, types[:2])
        out[name] = (ret, types[2:])
    return out


def mismatches(java, c):
    """Every difference between the Java declarations and the C definitions, as text."""
    bad = []
    for name in sorted(set(java) | set(c)):
        if name not in c:
            bad.append(f"{name}: declared native in ZarrHip.java, no JNI function")
            continue
        if name not in java:
            bad.append(f"{name}: JNI function without a native declaration")
            continue
        (jr, jp), (cr, cp) = java[name], c[name]
        if jr != cr:
            bad.append(f"{name}: returns {cr} in C, {jr} in Java")
        if len(jp) != len(cp):
            bad.append(f"{name}: {len(cp)} parameters in C, {len(jp)} in Java")
            continue
        for k, (a, b) in enumerate(zip(jp, cp)):
            if a != b:
                bad.append(f"{name}: parameter {k} is {b} in C, {a} in Java")
    return bad


@pytest.fixture(scope="module")
def sources():
    with open(JAVA) as f:
        java = f.read()
    with open(JNI_C) as f:
        csrc = f.read()
    return java, csrc


def test_every_native_matches_its_jni_function(sources):
    java, csrc = sources
    j, c = java_natives(java), c_natives(csrc)
    assert len(j) >= 10 and len(c) >= 10
    assert mismatches(j, c) == []


def test_mapping_examples():
    assert jni_type("long[]") == "jlongArray"
    assert jni_type("int[]") == "jintArray"
    assert jni_type("byte[][]") == "jobjectArray"
    assert jni_type("long[][]") == "jobjectArray"
    assert jni_type("String[]") == "jobjectArray"
    assert jni_type("Object") == "jobject"
    assert jni_type("String") == "jstring"
    assert jni_type("boolean") == "jboolean"


def test_checker_catches_a_swapped_array_type(sources):
    """The check is not vacuous: swapping one jlongArray for a jintArray in a prototype, or
    dropping a parameter, is reported."""
    java, csrc = sources
    j = java_natives(java)
    m = re.search(PREFIX + r"arrayReadFiles\s*\(", csrc)
    assert m
    i = csrc.index("jlongArray", m.end())
    swapped = csrc[:i] + "jintArray" + csrc[i + len("jlongArray"):]
    bad = mismatches(j, c_natives(swapped))
    assert bad == ["arrayReadFiles: parameter 0 is jintArray in C, jlongArray in Java"]
    k = csrc.index("jbyteArray jfill,", m.end())
    dropped = csrc[:k] + csrc[k + len("jbyteArray jfill,"):]
    bad = mismatches(j, c_natives(dropped))
    assert len(bad) == 1 and bad[0].startswith("arrayReadFiles: ") and "parameters" in bad[0]
