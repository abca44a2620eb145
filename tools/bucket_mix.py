"""Which stems share a partition bucket (top 10 bits of the 32-bit sort key)
with the hottest stems of bench.py's C2 batches, under a given stem-hash key.

The stem hash is the library's keyed SipHash-1-3 (rl_device.h StemHasher,
hash_key_of), restated here for this analysis only; the batches are
bench.py's four distinct C2 batches (rng 0xC2, Zipf(1.1) over 10M tenants).

    python tools/bucket_mix.py <hash_seed> [buckets=4]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ratelimit_amd import workloads as W  # noqa: E402

M = (1 << 64) - 1


def rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & M


def fmix(k):
    k ^= k >> 33
    k = (k * 0xff51afd7ed558ccd) & M
    k ^= k >> 33
    k = (k * 0xc4ceb9fe1a85ec53) & M
    return k ^ (k >> 33)


def hash_key(seed):
    return fmix(seed ^ 0x243F6A8885A308D3), fmix((seed + 0x13198A2E03707344) & M)


def stem_hash(key, s):
    k0, k1 = key
    v = [k0 ^ 0x736f6d6570736575, k1 ^ 0x646f72616e646f6d, k0 ^ 0x6c7967656e657261, k1 ^ 0x7465646279746573]

    def rnd():
        v[0] = (v[0] + v[1]) & M; v[1] = rotl(v[1], 13); v[1] ^= v[0]; v[0] = rotl(v[0], 32)
        v[2] = (v[2] + v[3]) & M; v[3] = rotl(v[3], 16); v[3] ^= v[2]
        v[0] = (v[0] + v[3]) & M; v[3] = rotl(v[3], 21); v[3] ^= v[0]
        v[2] = (v[2] + v[1]) & M; v[1] = rotl(v[1], 17); v[1] ^= v[2]; v[2] = rotl(v[2], 32)

    def word(m):
        v[3] ^= m
        rnd()
        v[0] ^= m

    n, i = len(s), 0
    while i + 8 <= n:
        word(int.from_bytes(s[i:i + 8], "little"))
        i += 8
    word(((n << 56) & M) | (int.from_bytes(s[i:], "little") if i < n else 0))
    v[2] ^= 0xff
    rnd(); rnd(); rnd()
    return (v[0] ^ v[1] ^ v[2] ^ v[3]) or 1


def main():
    key = hash_key(int(sys.argv[1]))
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rng = np.random.default_rng(0xC2)
    z = W.ZipfSampler(10_000_000, 1.1)
    for b in range(4):
        ten = z.sample(rng, 500_000)
        rng.integers(1, 9, 500_000)  # (the batch's hits, drawn by bench.py in between)
        t, c = np.unique(ten, return_counts=True)
        buckets = {}
        for tt, cc in zip(t, c):
            for suf in (b"_tier_sec_", b"_tier_min_"):
                sk = stem_hash(key, b"bench_tenant_t" + b"%010d" % tt + suf) >> 32
                buckets.setdefault(sk >> 22, []).append((int(cc), sk))
        top = sorted(((sum(x for x, _ in v), d, sorted(v, reverse=True)[:4]) for d, v in buckets.items()),
                     reverse=True)[:nb]
        for tot, d, keys in top:
            print("batch %d bucket %4d: %6d descriptors; largest stems %s" % (
                b, d, tot, ", ".join("%d (sort key %08x)" % (x, k) for x, k in keys)))


if __name__ == "__main__":
    main()
