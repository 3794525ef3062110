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
struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
    void* (*GetDirectBufferAddress)(JNIEnv*, jobject);
    jlong (*GetDirectBufferCapacity)(JNIEnv*, jobject);
    jstring (*NewStringUTF)(JNIEnv*, const char*);
    jobject (*NewDirectByteBuffer)(JNIEnv*, void*, jlong);
    void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);
};
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
"""

EXPECTED = ["open", "close", "lastError", "allocPinned", "freePinned", "verifyBatch", "requiredSigners", "txIds",
            "verifySignedTxBatch", "ftxVerify", "stxVerify", "uniqOpen", "uniqClose", "uniqSize", "uniqLastError",
            "uniqRebuild", "uniqCommitBatch"]


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
