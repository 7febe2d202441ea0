#!/usr/bin/env python3
"""Check operand-layout hypotheses for the gfx950 i8 MFMAs against tools/mfma_i8_layout output."""
import json
import sys

import numpy as np


def frags(words):
    return np.array(words, dtype=np.int32).view(np.int8).reshape(64, 16)


def check(d, a, b, M, K, kmap, cmap):
    A = np.zeros((M, K), np.int64)
    B = np.zeros((K, M), np.int64)
    for l in range(64):
        for j in range(16):
            r, k = kmap(l, j)
            A[r, k] = a[l, j]
            B[k, r] = b[l, j]
    C = A @ B
    got = np.zeros_like(C)
    regs = len(d) // 64
    for l in range(64):
        for r in range(regs):
            i, jj = cmap(l, r)
            got[i, jj] = d[regs * l + r]
    return np.array_equal(C, got)


def main():
    j = json.load(open(sys.argv[1]))
    a, b = frags(j["a"]), frags(j["b"])
    hyp32 = {
        "contig16": lambda l, jj: (l & 31, 16 * (l >> 5) + jj),
        "split8": lambda l, jj: (l & 31, 8 * (l >> 5) + jj if jj < 8 else 16 + 8 * (l >> 5) + jj - 8),
    }
    hyp16 = {
        "contig16": lambda l, jj: (l & 15, 16 * (l >> 4) + jj),
        "split8": lambda l, jj: (l & 15, 8 * (l >> 4) + jj if jj < 8 else 32 + 8 * (l >> 4) + jj - 8),
    }
    c32 = lambda l, r: ((r & 3) + 8 * (r >> 2) + 4 * (l >> 5), l & 31)
    c16 = lambda l, r: (4 * (l >> 4) + r, l & 15)
    res = {"32x32x32": {k: check(np.array(j["d32"]), a, b, 32, 32, f, c32) for k, f in hyp32.items()},
           "16x16x64": {k: check(np.array(j["d16"]), a, b, 16, 64, f, c16) for k, f in hyp16.items()}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
