"""ORACLE -- TEST INFRASTRUCTURE ONLY: RC4 as used by ugo/crypto.go:25-39.

rc4StreamCrypto builds a fresh crypto/rc4 cipher from the fixed key for every
packet (ugo/crypto.go:26,34), so every packet is XORed with the same keystream
prefix.  Plain KSA + PRGA restatement (Go's crypto/rc4 is standard RC4),
pinned by the classic published vectors in tests/test_rx_batch.py.
"""


def keystream(key: bytes, n: int) -> bytes:
    S = list(range(256))
    j = 0
    for i in range(256):
        j = (j + S[i] + key[i % len(key)]) & 0xFF
        S[i], S[j] = S[j], S[i]
    out = bytearray(n)
    i = j = 0
    for k in range(n):
        i = (i + 1) & 0xFF
        j = (j + S[i]) & 0xFF
        S[i], S[j] = S[j], S[i]
        out[k] = S[(S[i] + S[j]) & 0xFF]
    return bytes(out)


def xor_stream(key: bytes, data: bytes) -> bytes:
    ks = keystream(key, len(data))
    return bytes(a ^ b for a, b in zip(data, ks))
