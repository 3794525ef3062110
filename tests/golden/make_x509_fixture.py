#!/usr/bin/env python3
"""Extract the reference's own BouncyCastle-made ECDSA signatures into tests/golden/ref_x509_ecdsa.json.

Run here (in the build container, where /root/reference exists); the GPU box only reads the JSON.

The reference ships Java KeyStores holding X.509 certificate chains that Corda's X509Utilities signed
through BouncyCastle's ContentSigner with DEFAULT_TLS_SIGNATURE_SCHEME = Crypto.ECDSA_SECP256R1_SHA256
(node/src/main/kotlin/net/corda/node/utilities/X509Utilities.kt:44,278).  Each certificate is one
SHA256withECDSA signature:
    message   = the DER bytes of tbsCertificate            (RFC 5280 §4.1.1.1)
    signature = the BIT STRING payload of signatureValue   (DER ECDSA-Sig-Value, BC's StdDSAEncoder)
    key       = the issuer's SubjectPublicKeyInfo          (the chain link's parent certificate)
Those are exactly the inputs Crypto.doVerify(issuerKey, sigBytes, tbs) takes, and every link of a
chain the reference distributes verifies (the node loads these trust stores), so every record is a
reference-held VALID vector.

Only public certificate entries are read.  JKS layout (sun.security.provider.JavaKeyStore):
    u32 magic 0xFEEDFEED, u32 version (1|2), u32 count, then per entry
      u32 tag (1 private key, 2 trusted cert), UTF alias, u64 date,
      tag 1: u32 len + encrypted key (skipped), u32 chain length, chain certs
      tag 2: one cert
      cert: [version 2: UTF cert type] u32 len + DER
    and a 20-byte keyed SHA-1 trailer (not checked: it needs the store password).
"""
import base64
import json
import os
import struct
import sys

REF = "/root/reference"
SOURCES = [
    "node/src/main/resources/net/corda/node/internal/certificates/cordadevcakeys.jks",
    "node/src/main/resources/net/corda/node/internal/certificates/cordatruststore.jks",
    "samples/trader-demo/src/main/resources/certificates/truststore.jks",
    "samples/trader-demo/src/main/resources/certificates/sslkeystore.jks",
    "samples/attachment-demo/src/main/resources/certificates/truststore.jks",
    "samples/attachment-demo/src/main/resources/certificates/sslkeystore.jks",
    "config/dev/corda_dev_ca.cer",
]
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_x509_ecdsa.json")

OID_ECDSA_SHA256 = "1.2.840.10045.4.3.2"
OID_EC_PUBKEY = "1.2.840.10045.2.1"
CURVES = {"1.2.840.10045.3.1.7": "secp256r1", "1.3.132.0.10": "secp256k1"}
SCHEME = {"secp256r1": 3, "secp256k1": 2}


def jks_certs(blob):
    magic, version, count = struct.unpack(">III", blob[:12])
    if magic != 0xFEEDFEED or version not in (1, 2):
        raise ValueError("not a JKS store")
    p = 12
    out = []

    def utf():
        nonlocal p
        (n,) = struct.unpack(">H", blob[p:p + 2])
        s = blob[p + 2:p + 2 + n].decode("utf-8", "replace")
        p += 2 + n
        return s

    def cert():
        nonlocal p
        ctype = utf() if version == 2 else "X.509"
        (n,) = struct.unpack(">I", blob[p:p + 4])
        der = blob[p + 4:p + 4 + n]
        p += 4 + n
        return ctype, der

    for _ in range(count):
        (tag,) = struct.unpack(">I", blob[p:p + 4])
        p += 4
        alias = utf()
        p += 8
        if tag == 1:
            (n,) = struct.unpack(">I", blob[p:p + 4])
            p += 4 + n
            (chain,) = struct.unpack(">I", blob[p:p + 4])
            p += 4
            for k in range(chain):
                ctype, der = cert()
                out.append((alias, k, ctype, der))
        elif tag == 2:
            ctype, der = cert()
            out.append((alias, 0, ctype, der))
        else:
            raise ValueError("unknown JKS entry tag %d" % tag)
    return out


def tlv(b, p):
    """(tag, header_len, content_len) of the DER element at b[p]."""
    tag = b[p]
    L = b[p + 1]
    if L < 0x80:
        return tag, 2, L
    nb = L & 0x7F
    return tag, 2 + nb, int.from_bytes(b[p + 2:p + 2 + nb], "big")


def children(b, p):
    tag, h, n = tlv(b, p)
    q, end, out = p + h, p + h + n, []
    while q < end:
        t, hh, nn = tlv(b, q)
        out.append((q, t, hh, nn))
        q += hh + nn
    return out


def oid(b):
    first = b[0]
    parts = [first // 40, first % 40]
    v = 0
    for c in b[1:]:
        v = (v << 7) | (c & 0x7F)
        if not c & 0x80:
            parts.append(v)
            v = 0
    return ".".join(str(x) for x in parts)


def parse_cert(der):
    top = children(der, 0)
    (tp, _, th, tn), (ap, _, ah, an), (sp, st, sh, sn) = top
    tbs = der[tp:tp + th + tn]
    q0, _, h0, n0 = children(der, ap)[0]
    alg = oid(der[q0 + h0:q0 + h0 + n0])
    if st != 0x03 or der[sp + sh] != 0:
        raise ValueError("signatureValue is not a whole-byte BIT STRING")
    sig = der[sp + sh + 1:sp + sh + sn]
    f = children(der, tp)
    i = 1 if f[0][1] == 0xA0 else 0          # [0] EXPLICIT version present
    issuer = f[i + 2]
    subject = f[i + 4]
    spki = f[i + 5]
    name = lambda e: der[e[0]:e[0] + e[2] + e[3]]
    spki_der = name(spki)
    algid = children(spki_der, 0)[0]
    ids = children(spki_der, algid[0])
    key_alg = oid(spki_der[ids[0][0] + ids[0][2]:ids[0][0] + ids[0][2] + ids[0][3]])
    curve = None
    if len(ids) > 1 and ids[1][1] == 0x06:
        curve = CURVES.get(oid(spki_der[ids[1][0] + ids[1][2]:ids[1][0] + ids[1][2] + ids[1][3]]))
    return {"tbs": tbs, "sig_alg": alg, "sig": sig, "issuer": name(issuer), "subject": name(subject),
            "spki": spki_der, "key_alg": key_alg, "curve": curve}


def main():
    if not os.path.isdir(REF):
        sys.exit("needs /root/reference (run in the build container)")
    certs = []
    for rel in SOURCES:
        blob = open(os.path.join(REF, rel), "rb").read()
        if blob.startswith(b"-----BEGIN CERTIFICATE-----"):
            body = b"".join(l for l in blob.splitlines() if l and not l.startswith(b"-----"))
            blob = base64.b64decode(body)
        entries = jks_certs(blob) if blob[:4] == b"\xfe\xed\xfe\xed" else [("cer", 0, "X.509", blob)]
        for alias, k, ctype, der in entries:
            c = parse_cert(der)
            c.update(source=rel, alias=alias, chain_pos=k, der=der)
            certs.append(c)
    by_subject = {}
    for c in certs:
        by_subject.setdefault(c["subject"], []).append(c)
    # Several stores reuse one subject name with different keys (the dev CA is r1 in node/, k1 in the
    # samples), so a link's parent is the same-name certificate whose key verifies it.  That choice is
    # made with OpenSSL (tools/libcordagen.so), independent of oracle/, which the fixture then pins.
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tools"))
    import cordagen
    records, seen = [], set()
    for c in certs:
        if c["sig_alg"] != OID_ECDSA_SHA256:
            continue
        for parent in by_subject.get(c["issuer"], []):
            if parent["key_alg"] != OID_EC_PUBKEY or parent["curve"] not in SCHEME:
                continue
            key = (c["tbs"], c["sig"], parent["spki"])
            if key in seen:
                continue
            if cordagen.ossl_verify(parent["spki"], c["sig"], c["tbs"]) != 1:
                continue
            seen.add(key)
            records.append({
                "source": c["source"], "alias": c["alias"], "chain_pos": c["chain_pos"],
                "curve": parent["curve"], "scheme": SCHEME[parent["curve"]],
                "issuer_spki": parent["spki"].hex(), "tbs": c["tbs"].hex(), "sig_der": c["sig"].hex(),
                "self_signed": c["issuer"] == c["subject"],
            })
    doc = {
        "what": "reference-held SHA256withECDSA signatures (BouncyCastle-made X.509 chain links); each "
                "(issuer_spki, sig_der, tbs) is Crypto.doVerify(issuerKey, sig, tbs) == true",
        "generator": "tests/golden/make_x509_fixture.py",
        "reference_files": SOURCES,
        "cite": "node/src/main/kotlin/net/corda/node/utilities/X509Utilities.kt:44,278",
        "records": records,
    }
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print("%d certificates, %d distinct ECDSA chain links -> %s" % (len(certs), len(records), OUT))
    for r in records:
        print("  %-60s %-22s pos %d %s sig %d B tbs %d B%s" % (r["source"][-60:], r["alias"], r["chain_pos"], r["curve"],
                                                          len(r["sig_der"]) // 2, len(r["tbs"]) // 2,
                                                          " (self-signed)" if r["self_signed"] else ""))


if __name__ == "__main__":
    main()
