"""CPU: the JNI glue (jni/cordahip_jni.c) compiles against include/cordahip.h and links against
libcordahip.so, so every entry it binds (verifyBatch, requiredSigners, txIds, verifySignedTxBatch, ftxVerify,
stxVerify, uniq*) calls the C-ABI with the declared signatures.  No JDK exists in this image: the compile uses a
minimal stand-in for <jni.h> that declares only the JNIEnv functions the glue calls (a compile check of our own
glue; the JVM build in INTEGRATION.md uses the JDK's header)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

JNI_STUB = r"""
#pragma once
typedef int jint;
typedef long long jlong;
typedef unsigned char jboolean;
typedef jint jsize;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jlongArray;
typedef jobject jintArray;
typedef jobject jarray;
typedef double jdouble;
typedef jobject jdoubleArray;
struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
    void* (*GetDirectBufferAddress)(JNIEnv*, jobject);
    jlong (*GetDirectBufferCapacity)(JNIEnv*, jobject);
    jstring (*NewStringUTF)(JNIEnv*, const char*);
    jobject (*NewDirectByteBuffer)(JNIEnv*, void*, jlong);
    void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);
    jsize (*GetArrayLength)(JNIEnv*, jarray);
    void (*GetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, jint*);
    void (*SetDoubleArrayRegion)(JNIEnv*, jdoubleArray, jsize, jsize, const jdouble*);
};
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
"""

EXPECTED = ["open", "close", "lastError", "allocPinned", "freePinned", "verifyBatch", "requiredSigners", "txIds",
            "verifySignedTxBatch", "ftxVerify", "stxVerify", "uniqOpen", "uniqClose", "uniqSize", "uniqLastError",
            "uniqRebuild", "uniqCommitBatch", "groupOpen", "groupClose", "groupLastError", "groupSize", "groupMember",
            "groupVerifyBatch", "groupTxIds", "groupVerifySignedTxBatch", "groupFtxVerify", "groupStxVerify",
            "groupUniqOpen", "groupUniqClose", "groupUniqSize", "groupUniqLastError", "groupUniqRebuild",
            "groupUniqCommitBatch", "groupLastStats", "uniqLastRounds"]


def test_jni_glue_compiles_and_links(tmp_path):
    lib = os.path.join(ROOT, "corda_amd", "libcordahip.so")
    if not os.path.exists(lib):
        pytest.skip("libcordahip.so not built")
    inc = tmp_path / "inc"
    inc.mkdir()
    (inc / "jni.h").write_text(JNI_STUB)
    out = tmp_path / "libcordahip_jni.so"
    r = subprocess.run(["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter", "-shared",
                        "-fPIC", "-I", str(inc), "-I", os.path.join(ROOT, "include"), "-o", str(out),
                        os.path.join(ROOT, "jni", "cordahip_jni.c"), "-L", os.path.join(ROOT, "corda_amd"),
                        "-lcordahip", "-Wl,--no-undefined", "-Wl,-rpath," + os.path.join(ROOT, "corda_amd")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    syms = subprocess.check_output(["nm", "-D", "--defined-only", str(out)], text=True)
    for name in EXPECTED:
        assert "Java_net_corda_core_internal_gpu_CordaHip_" + name in syms, name


def test_kotlin_natives_match_the_glue():
    """Every `external fun` of CordaHip.kt has a JNI function in the glue, and the reverse."""
    import re
    kt = open(os.path.join(ROOT, "jni", "CordaHip.kt")).read()
    c = open(os.path.join(ROOT, "jni", "cordahip_jni.c")).read()
    ext = set(re.findall(r"external fun (\w+)\(", kt))
    glue = set(re.findall(r"CLS\((\w+)\)", c)) - {"name"}   # minus the #define
    assert ext == glue == set(EXPECTED)


# Kotlin stdlib functions and language features newer than the reference's Kotlin 1.1.50
# (/root/reference/constants.properties:2, kotlin-stdlib-jre8 in core/build.gradle:28): the binding must compile there.
POST_11 = {
    "sumOf": "1.4", "zipWithNext": "1.2", "chunked": "1.2", "windowed": "1.2", "buildList": "1.6", "buildMap": "1.6",
    "ifEmpty": "1.3", "ifBlank": "1.3", "removeLast": "1.4", "removeFirst": "1.4", "lowercase": "1.5",
    "uppercase": "1.5", "maxOrNull": "1.4", "minOrNull": "1.4", "maxByOrNull": "1.4", "minByOrNull": "1.4",
    "associateWith": "1.3", "runCatching": "1.3", "firstNotNullOf": "1.5", "orEmpty() ": "-", "shuffled": "1.2",
    "toUByte": "1.3", "toUInt": "1.3", "readText(": "-", "scan(": "1.4", "runningFold": "1.4", "onEachIndexed": "1.4",
    "flatMapIndexed": "1.4", "reduceOrNull": "1.4", "randomOrNull": "1.4", "fill(": "1.2", "contentToString": "1.1.60",
    "mapNotNullTo": "-", "getValue(": "1.1", "digitToInt": "1.5", "fold(": "1.0", "also": "1.1", "takeIf": "1.1",
}
DENY = [k for k, v in POST_11.items() if v not in ("1.0", "1.1", "-")]
KT = ["BatchSignatureVerifier.kt", "BatchFilteredTransactionVerifier.kt", "CordaHip.kt", "GpuUniquenessProvider.kt"]


def _kt(name):
    src = open(os.path.join(ROOT, "jni", name)).read()
    import re
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


@pytest.mark.parametrize("name", KT)
def test_kotlin_binding_uses_the_1_1_stdlib_only(name):
    """No stdlib call or language feature newer than Kotlin 1.1 (an explicit deny-list), so the binding compiles with
    the reference's toolchain."""
    import re
    src = _kt(name)
    for sym in DENY:
        pat = r"\b" + re.escape(sym.rstrip("(")) + (r"\s*\(" if sym.endswith("(") else r"\b")
        assert not re.search(r"\." + pat if not sym.endswith("(") else pat, src), (name, sym, POST_11[sym])
    assert not re.search(r"\.code\b", src), (name, ".code (1.5)")
    assert not re.search(r"when\s*\(\s*val\b", src), (name, "when subject val (1.3)")
    assert not re.search(r"\bfun\s+interface\b", src), (name, "fun interface (1.4)")
    assert not re.search(r",\s*\n\s*[)\]>]", src), (name, "trailing comma (1.4)")
    assert not re.search(r"\bsealed\s+interface\b|@JvmInline|\bvalue\s+class\b", src), name


@pytest.mark.parametrize("name", ["BatchSignatureVerifier.kt", "BatchFilteredTransactionVerifier.kt"])
def test_every_device_call_has_a_jvm_fallback(name):
    """Each library call of the verifiers goes through GpuHandle.ok: CHIP_E_DEVICE / CHIP_E_NOMEM send that batch to
    the JVM path (the JCA engines / the reference's own checks), only CHIP_E_ARG throws.  No bare check(rc == 0)."""
    import re
    src = _kt(name)
    assert "check(rc == 0)" not in src
    calls = [m.start() for m in re.finditer(r"val rc = ", src)]
    assert len(calls) >= (4 if name.startswith("BatchSig") else 1)
    for at in calls:
        tail = src[at:at + 2000]
        m = re.search(r"if \(!gpu\.ok\(rc, \"\w+\"\)\)", tail)
        assert m, (name, src[at:at + 120])
        after = tail[m.end():m.end() + 200].lstrip()
        assert after.startswith("return") or after.startswith("//") or after.startswith("{"), (name, after[:80])


def test_gpu_handle_policy():
    """GpuHandle.ok: 0 true; CHIP_E_DEVICE / CHIP_E_NOMEM false (fallback, counted); anything else throws."""
    src = _kt("CordaHip.kt")
    body = src[src.index("fun ok(rc: Int"):]
    body = body[:body.index("override fun close")]
    assert "rc == CordaHip.E_DEVICE || rc == CordaHip.E_NOMEM" in body and "return false" in body
    assert "throw IllegalStateException" in body
    assert "const val E_DEVICE = -2" in src and "const val E_NOMEM = -3" in src and "const val E_ARG = -1" in src
