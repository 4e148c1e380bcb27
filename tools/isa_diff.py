"""Compare the device assembly of two builds kernel by kernel (hipcc --cuda-device-only -S output):
which kernels' instruction streams differ.  Used to check that a source clean-up (knobs folded to
constants, dead A/B paths removed) leaves the product's machine code unchanged.

    python3 tools/isa_diff.py before.s after.s
"""
import re
import sys


def kernels(path):
    out, cur, body = {}, None, []
    for line in open(path):
        m = re.match(r"^([_A-Za-z][\w$.]*):\s*(;.*)?$", line)
        if m and not m.group(1).startswith(".L"):
            if cur:
                out[cur] = body
            cur, body = m.group(1), []
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            out[cur] = body
            cur, body = None, []
            continue
        s = line.split(";")[0].strip()
        if not s or s.startswith(".") and not s.startswith(".LBB"):
            continue
        body.append(re.sub(r"\.LBB\d+_(\d+)", r".LBB_\1", s))
    if cur:
        out[cur] = body
    return out


a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
same = diff = 0
for k in sorted(set(a) | set(b)):
    if k not in a or k not in b:
        print(("only in after: " if k in b else "only in before: ") + k)
        diff += 1
    elif a[k] != b[k]:
        print(f"differs: {k} ({len(a[k])} -> {len(b[k])} instructions)")
        diff += 1
    else:
        same += 1
print(f"{same} kernels identical, {diff} differ")
