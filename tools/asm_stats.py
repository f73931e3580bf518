"""Per-kernel code statistics of a hipcc --cuda-device-only -S listing:
instruction count, VGPR/SGPR counts, scratch. Used to check that a source
change leaves a hot kernel's code unchanged (e.g. a new template instance
beside it).  Usage: python tools/asm_stats.py file.s [file.s ...]
"""
import re
import sys


def stats(path):
    text = open(path).read().splitlines()
    out, cur, n = {}, None, 0
    for line in text:
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            cur, n = m.group(1), 0
            continue
        if cur and line.startswith("\ts_endpgm"):
            out[cur] = {"insts": n + 1}
            cur = None
            continue
        if cur and line.startswith("\t") and not line.startswith("\t.") and not line.strip().startswith(";"):
            n += 1
    meta = re.findall(r"\.name:\s+(_Z\S+)\n(?:.*\n)*?\s+\.sgpr_count:\s+(\d+)\n(?:.*\n)*?\s+\.vgpr_count:\s+(\d+)",
                      "\n".join(text))
    for name, s, v in meta:
        out.setdefault(name, {})["sgpr"] = int(s)
        out[name]["vgpr"] = int(v)
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        for k, v in sorted(stats(p).items()):
            print(f"{p.split('/')[-1]:10s} {v.get('insts', 0):6d} insts  v{v.get('vgpr', 0):4d} s{v.get('sgpr', 0):4d}  {k}")
