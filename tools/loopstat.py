"""Instruction mix / order of the loops of one kernel in a hipcc -save-temps .s file.
usage: python tools/loopstat.py <file.s> <kernel-symbol-substring> [--seq]"""
import collections
import re
import sys

src, sym = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + sym + r"\w*:", l) or l.startswith(sym + ":"))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
body = lines[start:end]
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
for i, l in enumerate(body):
    m = re.search(r"s_(?:c)?branch\w*\s+(\.LBB\w+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        seg = [x.split()[0] for x in body[labels[m.group(1)] + 1:i] if x.strip() and not x.strip().startswith(";") and not x.startswith(".")]
        c = collections.Counter(seg)
        print(f"loop {m.group(1)}: {len(seg)} instrs, mfma {sum(v for k, v in c.items() if 'mfma' in k)}")
        print("   " + ", ".join(f"{k} {v}" for k, v in c.most_common(16)))
        if "--seq" in sys.argv:
            abbrev = {"v_mfma_f32_32x32x16_bf16": "M", "v_mfma_f32_16x16x32_bf16": "m", "v_exp_f32_e32": "E", "v_fma_f32": "F", "v_accvgpr_read_b32": "R",
                      "v_accvgpr_write_b32": "w", "v_cvt_pk_bf16_f32": "C", "v_add_f32_e64": "A", "v_add_f32_e32": "A",
                      "v_pk_add_f32": "P", "ds_read_b128": "D", "ds_write_b128": "X", "v_mov_b32_e32": "v",
                      "s_waitcnt": "W", "global_load_dwordx4": "G", "s_barrier": "|B|", "s_nop": "n"}
            print("   " + " ".join(abbrev.get(x, "." ) for x in seg))
