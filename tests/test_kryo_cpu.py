"""CPU: the Kryo 4.0.0 SignableData restatement (corda_amd/kryo.py, include/corda/verify.hpp kryo::).

PARITY UNPINNED: the reference holds no serialized SignableData bytes and no JVM runs here.  These
tests pin the restatement's own rules: write -> read round trips, the documented byte layout of
each Kryo construct, the fixed id offset the fused tx-verify templates rely on, and Python == C++.
"""
import os
import subprocess

import pytest

from corda_amd import crypto as C
from corda_amd import kryo as K

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
METAS = [(1, 2), (1, 3), (1, 4), (2, 4), (63, 4), (64, 4), (1000, 3), (-1, 4)]


def test_primitives():
    assert K.varint(0) == b"\x00" and K.varint(127) == b"\x7f" and K.varint(128) == b"\x80\x01"
    assert K.varint(1, False) == b"\x02" and K.varint(-1, False) == b"\x01" and K.varint(64, False) == b"\x80\x01"
    assert K.string("ab") == b"a\xe2"
    assert K.string("") == b"\x81"
    assert K.string("a")[0] & 0x80   # 1-char strings take the UTF-8 path
    assert K.chunked(b"xyz") == b"\x03xyz\x00"
    assert K.chunked(bytes(1500)) == b"\x80\x08" + bytes(1024) + b"\xdc\x03" + bytes(476) + b"\x00"


def test_layout_of_signable_data():
    tx = bytes(range(32))
    b = K.signable_data(tx, 1, 4)
    assert b.startswith(b"corda\x00\x00\x01\x01\x00net.corda.core.crypto.SignableDat\xe1\x01\x02")
    # field names of the three CompatibleFieldSerializer headers, sorted by EXTENDED cached name
    for name in (b"SignableData.signatureMetadat\xe1SignableData.txI\xe4",
                 b"SignatureMetadata.platformVersio\xeeSignatureMetadata.schemeNumberI\xc4",
                 b"\x01\x01net.corda.core.crypto.SecureHash$SHA25\xb6\x01\x01OpaqueBytes.byte\xf3"):
        assert name in b
    # metadata ints are zig-zag varints inside their own chunked fields; every inner flush also flushes
    # the enclosing field's OutputChunked (Output.flush -> parent.flush): the signatureMetadata field
    # is chunk(NOT_NULL, header, 01 02) chunk(00 01 08) chunk(00) 00
    assert b"\x45\x01\x02SignatureMetadata." in b
    assert b"\x01\x02\x03\x00\x01\x08\x01\x00\x00" in b
    # the id: NOT_NULL, length + 1, 32 bytes, then the inner end marker as its own chunk and the outer
    assert b.endswith(b"\x01\x21" + tx + b"\x01\x00\x00")
    assert len(b) == 269


@pytest.mark.parametrize("pv,sch", METAS)
def test_round_trip_and_template(pv, sch):
    tx = bytes((7 * i + pv) & 0xFF for i in range(32))
    b = K.signable_data(tx, pv, sch)
    assert K.parse_signable_data(b) == (tx, pv, sch)
    t, at = K.signable_data_template(pv, sch)
    assert t[:at] + tx + t[at:] == b
    assert C.signable_data_bytes(tx, C.SignatureMetadata(pv, sch)) == b


def test_parser_rejects_other_layouts():
    b = K.signable_data(bytes(32), 1, 4)
    with pytest.raises(K.KryoException):
        K.parse_signable_data(b"cordb" + b[5:])
    with pytest.raises(K.KryoException):
        K.parse_signable_data(b + b"\x00")
    with pytest.raises(K.KryoException):
        K.parse_signable_data(b[:-3])
    with pytest.raises(K.KryoException):
        K.signable_data(bytes(31), 1, 4)


def test_cpp_restatement_matches(tmp_path):
    exe = tmp_path / "kryo_bytes"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                        "-o", str(exe), os.path.join(ROOT, "tests", "cpp", "kryo_bytes.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    args = [str(x) for m in METAS for x in m]
    out = subprocess.check_output([str(exe)] + args, text=True).split()
    tx = bytes(range(32))
    assert out == [K.signable_data(tx, pv, sch).hex() for pv, sch in METAS]
