"""Count the instructions of each kernel's innermost hot loop in a device .s file
(hipcc --cuda-device-only -S).  Usage: isa_count.py file.s [kernel-substring ...]"""
import collections
import re
import sys


def loops(body):
    lines = [l.strip() for l in body.split("\n")]
    out = []
    for i, l in enumerate(lines):
        m = re.match(r"(\.LBB\d+_\d+):", l)
        if not m:
            continue
        lab = m.group(1)
        for j in range(i + 1, len(lines)):
            if lines[j].startswith("s_cbranch") and lines[j].split()[-1] == lab:
                seg = [x for x in lines[i + 1:j] if x and not x.startswith((".", ";", "//"))]
                out.append((lab, seg))
                break
    return out


def main():
    s = open(sys.argv[1]).read()
    want = sys.argv[2:]
    for m in re.finditer(r"^(_Z\w+):", s, re.M):
        name = m.group(1)
        if want and not any(w in name for w in want):
            continue
        body = s[m.end():]
        body = body[:body.index(".Lfunc_end")]
        for lab, seg in loops(body):
            c = collections.Counter(x.split()[0] for x in seg)
            print(f"{name} {lab}: {len(seg)} instrs", dict(c.most_common(14)))


if __name__ == "__main__":
    main()
