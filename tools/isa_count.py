"""Instruction mix of the kernels in a hipcc --save-temps device .s file.

    python tools/isa_count.py <file.s> [kernel-name-substring]
"""
import collections
import re
import sys


def main() -> None:
    s = open(sys.argv[1]).read()
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    for fn in re.findall(r"^(_Z\S+):", s, re.M):
        if pat not in fn or fn.endswith(".const"):
            continue
        body = s.split(fn + ":", 1)[1].split(".Lfunc_end", 1)[0]
        c = collections.Counter()
        for line in body.splitlines():
            line = line.strip()
            if not line or line.startswith((".", ";", "_")) or line.endswith(":"):
                continue
            c[line.split()[0]] += 1
        print(fn[:60], "instructions:", sum(c.values()))
        print("  ", c.most_common(30))


if __name__ == "__main__":
    main()
