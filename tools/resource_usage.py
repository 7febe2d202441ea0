#!/usr/bin/env python3
"""Per-kernel registers, spills, LDS and occupancy from hipcc -Rpass-analysis=kernel-resource-usage
remarks (stderr of a build), optionally against a second build's remarks.

  hipcc ... -Rpass-analysis=kernel-resource-usage -o /tmp/x.so csrc/sr_route.hip 2> new.txt
  python tools/resource_usage.py new.txt [old.txt]
"""
import re
import subprocess
import sys

KEYS = ("TotalSGPRs", "VGPRs", "SGPRs Spill", "VGPRs Spill", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]",
        "LDS Size [bytes/block]")


def parse(path):
    out, cur = {}, None
    for line in open(path):
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark:\s+(.+?): (\d+) \[", line)
        if m and cur and m.group(1) in KEYS:
            out[cur][m.group(1)] = int(m.group(2))
    return out


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        return r.stdout.splitlines()
    except (OSError, subprocess.CalledProcessError):
        return list(names)


def main():
    new = parse(sys.argv[1])
    old = parse(sys.argv[2]) if len(sys.argv) > 2 else {}
    names = sorted(new)
    for n, d in zip(names, demangle(names)):
        a, b = old.get(n), new[n]
        cols = " ".join(f"{k.split()[0][:5]}={b.get(k)}" for k in KEYS)
        mark = "" if not old else (" (new)" if a is None else ("" if a == b else " was " + " ".join(
            f"{k.split()[0][:5]}={a.get(k)}" for k in KEYS if a.get(k) != b.get(k))))
        print(f"{d[:100]:100s} {cols}{mark}")


if __name__ == "__main__":
    main()
