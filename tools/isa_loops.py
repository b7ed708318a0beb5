"""Static instruction accounting of one kernel in a hipcc --save-temps .s (built with -gline-tables-only):
per loop (back-edge) the instruction mix of its body and the source lines it comes from.

  python tools/isa_loops.py FILE.s KERNEL_SYMBOL [--min 20]
"""
import collections
import re
import sys


def parse(path, kern):
    s = open(path).read()
    start = s.index(kern + ":")
    end = s.index(".Lfunc_end", start)
    files = dict(re.findall(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s, flags=re.M))
    blocks, cur, lab, loc = [], None, {}, ("?", 0)
    for ln in s[start:end].split("\n"):
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            cur = {"name": m.group(1), "ins": []}
            blocks.append(cur)
            lab[m.group(1)] = len(blocks) - 1
            continue
        if cur is None:
            cur = {"name": "entry", "ins": []}
            blocks.append(cur)
        t = ln.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if m:
            loc = (files.get(m.group(1), m.group(1)), int(m.group(2)))
            continue
        if not t or t.startswith((".", ";", "//")):
            continue
        cur["ins"].append((t, loc))
    return blocks, lab


def kind(op):
    if op.startswith(("v_fma_f64", "v_fmac_f64", "v_mul_f64", "v_add_f64", "v_rcp_f64", "v_div", "v_ldexp_f64",
                      "v_max_f64", "v_min_f64", "v_frexp", "v_fract_f64", "v_trig", "v_rndne_f64", "v_sqrt_f64",
                      "v_cmp_class_f64")):
        return "f64"
    if op.startswith("v_cmp") or op.startswith("v_cndmask"):
        return "cmp/sel"
    if op.startswith(("v_mov", "v_readlane", "v_writelane", "v_readfirstlane")):
        return "mov"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, kern = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 20
    blocks, lab = parse(path, kern)
    loops = set()
    for j, b in enumerate(blocks):
        for t, _ in b["ins"]:
            m = re.match(r"s_(cbranch_\w+|branch)\s+(\.LBB\S+)", t)
            if m and m.group(2) in lab and lab[m.group(2)] <= j:
                loops.add((lab[m.group(2)], j))
    tot = collections.Counter(kind(t.split()[0]) for b in blocks for t, _ in b["ins"])
    print("whole kernel:", dict(tot))
    for i, j in sorted(loops):
        c, lines = collections.Counter(), collections.Counter()
        for b in blocks[i:j + 1]:
            for t, loc in b["ins"]:
                k = kind(t.split()[0])
                c[k] += 1
                if k not in ("salu", "wait"):
                    lines[f"{loc[0]}:{loc[1]}"] += 1
        n = sum(c.values())
        if n < mn:
            continue
        valu = c["f64"] + c["cmp/sel"] + c["mov"] + c["valu_other"]
        print(f"{blocks[i]['name']}..{blocks[j]['name']} blocks={j - i + 1} n={n} valu={valu} " +
              " ".join(f"{k}={v}" for k, v in sorted(c.items())))
        print("    top lines:", ", ".join(f"{k}({v})" for k, v in lines.most_common(6)))


if __name__ == "__main__":
    main()
