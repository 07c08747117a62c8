# Developer tool: static instruction mix per kernel of a hipcc --save-temps .s file, with the
# per-loop breakdown of scripts/loops.py for one kernel.  Used to check that writing the fused
# multiply-adds out explicitly (-ffp-contract=off) keeps the instruction counts:
#   python3 scripts/isa_counts.py file.s [kernel-substring]
import re
import sys


def kernels(asm):
    for m in re.finditer(r'^(_Z\w+):[^\n]*$(.*?)^\.Lfunc_end', asm, re.S | re.M):
        yield m.group(1), m.group(2).splitlines()


def mix(lines):
    ins = [x.split()[0] for x in lines if x.strip() and not x.strip().startswith((';', '.')) and not x.strip().endswith(':')]
    return {
        "total": len(ins),
        "valu": sum(1 for x in ins if x.startswith('v_')),
        "fma64": sum(1 for x in ins if re.match(r'v_fma(c)?_f64', x)),
        "mul64": sum(1 for x in ins if x.startswith('v_mul_f64')),
        "add64": sum(1 for x in ins if x.startswith('v_add_f64')),
        "dpp": sum(1 for x in ins if 'dpp' in x),
    }


def loops(body):
    labels = {}
    for i, l in enumerate(body):
        mm = re.match(r'^(\.LBB\d+_\d+):', l)
        if mm:
            labels[mm.group(1)] = i
    out = []
    for i, l in enumerate(body):
        mm = re.search(r's_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)', l)
        if mm:
            t = mm.group(1) or mm.group(2)
            if t in labels and labels[t] < i:
                out.append((t, labels[t], i, mix(body[labels[t]:i + 1])))
    return out


if __name__ == "__main__":
    asm = open(sys.argv[1]).read()
    sel = sys.argv[2] if len(sys.argv) > 2 else None
    for name, body in kernels(asm):
        if sel and sel not in name:
            continue
        m = mix(body)
        print(f"{name[:70]:70s} " + " ".join(f"{k} {v}" for k, v in m.items()))
        if sel:
            for t, a, b, lm in loops(body):
                print(f"   loop {t} {a}-{b}: " + " ".join(f"{k} {v}" for k, v in lm.items()))
