"""Instruction-class histogram of the matrix-core factor walk's step loop (developer tool, no GPU):
    python3 scripts/isa_classes.py [source.hip ...]
compiles each source (default: the in-tree qsp_solver.hip) with the library's flags to assembly, takes
the headline kernel qp_step_kernel<1, false, true, true>, finds the loops that issue v_mfma_f64 and
prints, per walk step (a loop iteration divided by the MFMAs per step, eleven), the instructions by
class.  The loop body is straight-line code between its label and its back branch, so the static
counts are the issued counts per step."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KERNEL = "_ZN3qsp14qp_step_kernelILi1ELb0ELb1ELb1EEEvNS_9SolveArgsEi"
CLASSES = [
    ("mfma", lambda x: x.startswith("v_mfma")),
    ("fp64 arith", lambda x: re.match(r"v_(fma|fmac|mul|add|rcp|div\w*|ldexp|frexp\w*|max|min)_f64", x)),
    ("mov/dpp", lambda x: x.startswith("v_mov") or "dpp" in x),
    ("permlane", lambda x: x.startswith("v_permlane")),
    ("cndmask", lambda x: x.startswith("v_cndmask")),
    ("v_cmp", lambda x: x.startswith("v_cmp")),
    ("accvgpr", lambda x: x.startswith("v_accvgpr")),
    ("readlane/writelane", lambda x: x.startswith(("v_readlane", "v_writelane", "v_readfirstlane"))),
    ("int/address valu", lambda x: x.startswith("v_")),
    ("ds_read", lambda x: x.startswith("ds_read")),
    ("ds_write", lambda x: x.startswith("ds_write")),
    ("salu/branch", lambda x: x.startswith("s_")),
]


def classify(ins):
    out = {k: 0 for k, _ in CLASSES}
    other = 0
    for x in ins:
        for k, f in CLASSES:
            if f(x):
                out[k] += 1
                break
        else:
            other += 1
    out["other"] = other
    return out


def walk_loops(asm):
    m = re.search(r"^" + KERNEL + r":[^\n]*$(.*?)^\.Lfunc_end", asm, re.S | re.M)
    body = m.group(1).splitlines()
    labels = {}
    for i, l in enumerate(body):
        mm = re.match(r"^(\.LBB\d+_\d+):", l)
        if mm:
            labels[mm.group(1)] = i
    for i, l in enumerate(body):
        mm = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", l)
        if not mm:
            continue
        t = mm.group(1) or mm.group(2)
        if t not in labels or labels[t] >= i:
            continue
        ins = [x.split()[0] for x in body[labels[t]:i + 1]
               if x.strip() and not x.strip().startswith((";", ".")) and not x.strip().endswith(":")]
        nm = sum(1 for x in ins if x.startswith("v_mfma"))
        if nm:
            yield t, nm, ins


def main():
    from uclv_qs_pushing_matlab_amd.build import FLAGS
    flags = [f for f in FLAGS if f not in ("-shared", "-fPIC")]
    srcs = sys.argv[1:] or [os.path.join(ROOT, "uclv_qs_pushing_matlab_amd", "csrc", "qsp_solver.hip")]
    for src in srcs:
        with tempfile.TemporaryDirectory() as d:
            s = os.path.join(d, "k.s")
            subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", *flags, "-I", os.path.join(ROOT, "include"),
                                   "-I", os.path.join(ROOT, "uclv_qs_pushing_matlab_amd", "csrc"), "--cuda-device-only",
                                   "-S", src, "-o", s])
            asm = open(s).read()
        print(f"== {src}")
        for t, nm, ins in walk_loops(asm):
            steps = nm / 11
            c = classify(ins)
            print(f"  loop {t}: {len(ins)} instructions, {nm} MFMA = {steps:g} steps; per step:")
            print("    " + ", ".join(f"{k} {v / steps:.1f}" for k, v in c.items() if v))


if __name__ == "__main__":
    main()
