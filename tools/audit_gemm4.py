"""Audit the 4-wave GEMM's hand-placed accumulator file and inline-asm MFMAs in a -save-temps assembly file:
  1. no compiler-generated instruction references an AGPR (the accumulators are pinned in a[0:255]);
  2. no VALU write to an MFMA A/B operand VGPR within the 4 instructions before an inline-asm MFMA (hipcc does
     not pad hazards for asm consumers);
  3. no scratch (private segment) use.
python tools/audit_gemm4.py path/to/gemm-hip-amdgcn-amd-amdhsa-gfx950.s"""
import re
import sys


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def audit(path):
    text = open(path).read().split("\n")
    bad = 0
    starts = [i for i, l in enumerate(text) if re.match(r"^_ZN12_GLOBAL__N_1\d+gemm4_kernel_\w*:", l)]
    for st in starts:
        en = next(i for i in range(st, len(text)) if text[i].startswith(".Lfunc_end"))
        name = text[st].split(":")[0]
        body = text[st:en]
        inasm, recent, n_mfma = False, [], 0
        for l in body:
            t = l.split(";")[0].strip()
            if ";;#ASMSTART" in l:
                inasm = True
                continue
            if ";;#ASMEND" in l:
                inasm = False
                continue
            if not t or t.startswith("."):
                continue
            op = t.split()[0]
            if "scratch_" in op:
                print(f"{name}: scratch access: {t}"); bad += 1
            if not inasm:
                if re.search(r"\ba\[\d+|\ba\d+\b", t) and "accvgpr" in op or op.startswith("v_accvgpr"):
                    print(f"{name}: compiler AGPR use: {t}"); bad += 1
                if op.startswith("v_") and not op.startswith(("v_readlane", "v_readfirstlane", "v_cmp")):
                    dst = t[len(op):].split(",")[0].strip()
                    recent.append(regs(dst))
                else:
                    recent.append(set())
                recent = recent[-4:]
            elif op.startswith("v_mfma"):
                n_mfma += 1
                ops = [x.strip() for x in t[len(op):].split(",")]
                used = regs(ops[1]) | regs(ops[2])
                for w in recent:
                    if w & used:
                        print(f"{name}: VALU write to an MFMA operand right before it: {sorted(w & used)} in {t}")
                        bad += 1
                recent = []
        print(f"{name[:60]}...: {n_mfma} asm MFMAs checked")
    return bad


if __name__ == "__main__":
    n = audit(sys.argv[1])
    print("AUDIT", "FAILED" if n else "OK", n)
    sys.exit(1 if n else 0)
