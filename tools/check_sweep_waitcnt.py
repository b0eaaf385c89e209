"""Check the partitioned sweep's hand-counted LDS-DMA waits in the built ISA (ADVICE r04:
sweep.hip wait_vm<N> is right only while the compiler emits exactly the vector-memory
instructions the count assumes after the `global_load_lds` of the chain maps).

Compiles sweep.hip for gfx950 to assembly and runs a forward dataflow over every kernel's basic
blocks (branches and loop back-edges followed to a fixpoint; a merge keeps the worst path).  After an LDS
DMA (`global_load_lds_*` / `buffer_load_* ... lds`) it counts the vector-memory instructions
issued behind it; an `s_waitcnt vmcnt(N)` with N <= that count retires the DMA (vmcnt completes
in issue order).  Every LDS read (`ds_read*`) met while a DMA is still outstanding is reported
-- such a read could see LDS bytes the DMA has not written yet.

usage: python tools/check_sweep_waitcnt.py [--asm FILE] [--define HH_SWEEP_WAIT_ALL]
exit status 1 if any read is uncovered."""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "helmholtz_preconditioner_amd", "csrc")
VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)")
DMA = re.compile(r"^(global_load_lds_|buffer_load_\w+.*\blds\b)")
WAIT = re.compile(r"^s_waitcnt\b.*vmcnt\((\d+)\)")


def compile_asm(defines):
    out = os.path.join(tempfile.mkdtemp(), "sweep.s")
    cmd = [os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), "-O3", "-std=c++17",
           "--offload-arch=gfx950", "--cuda-device-only", "-S", "-I/opt/rocm/include",
           "-I" + os.path.join(ROOT, "include"), os.path.join(CSRC, "sweep.hip"), "-o", out]
    cmd += [f"-D{d}" for d in defines]
    subprocess.run(cmd, check=True, cwd=CSRC)
    return out


def blocks_of(lines):
    """basic blocks [(label, [insns], [successor labels])] of one function's body"""
    blocks, cur, body = [], "entry", []
    for ln in lines:
        m = re.match(r"^(\.LBB[\w]+):", ln)
        if m:
            blocks.append([cur, body])
            cur, body = m.group(1), []
        else:
            body.append(ln)
    blocks.append([cur, body])
    out = []
    for k, (lab, ins) in enumerate(blocks):
        succ = []
        last = ins[-1] if ins else ""
        for op in ins:
            t = re.match(r"^s_(cbranch_\w+|branch)\s+(\.LBB\w+)", op)
            if t:
                succ.append(t.group(2))
        if not (last.startswith("s_branch") or last.startswith("s_endpgm") or
                last.startswith("s_setpc")) and k + 1 < len(blocks):
            succ.append(blocks[k + 1][0])
        out.append((lab, ins, succ))
    return out


def transfer(state, ins, report=None, fn=None):
    """state: None (no DMA outstanding) or the number of vector-memory ops behind the oldest
    outstanding DMA (worst case over paths)"""
    for i, op in enumerate(ins):
        if DMA.match(op):
            state = 0 if state is None else min(state, 0)
        elif VMEM.match(op) and state is not None:
            state += 1
        w = WAIT.match(op)
        if w and state is not None and int(w.group(1)) <= state:
            state = None
        if op.startswith("ds_read") and state is not None and report is not None:
            report.append((fn, op, state))
    return state


def scan(path):
    funcs, cur = {}, None
    for raw in open(path):
        line = raw.split(";")[0].strip()
        m = re.match(r"^([A-Za-z_][\w.$]*):", raw)
        if m and not m.group(1).startswith(".L"):
            cur = m.group(1)
            funcs[cur] = []
            continue
        if raw.startswith(".Lfunc_end"):
            cur = None
            continue
        if cur and line and (not line.startswith(".") or re.match(r"^\.LBB\w+:", line)):
            funcs[cur].append(line)
    report = []
    ndma = 0
    worst = lambda a, b: b if a is None else (a if b is None else min(a, b))  # noqa: E731
    for fn, lines in funcs.items():
        bl = blocks_of(lines)
        ndma += sum(1 for _, ins, _ in bl for op in ins if DMA.match(op))
        idx = {lab: k for k, (lab, _, _) in enumerate(bl)}
        IN = {lab: "unreached" for lab, _, _ in bl}
        IN["entry"] = None
        changed = True
        while changed:  # forward dataflow to a fixpoint (merge: the worst path)
            changed = False
            for lab, ins, succ in bl:
                if IN[lab] == "unreached":
                    continue
                o = transfer(IN[lab], ins)
                for sc in succ:
                    if sc not in idx:
                        continue
                    new = o if IN[sc] == "unreached" else worst(IN[sc], o)
                    if new != IN[sc]:
                        IN[sc], changed = new, True
        for lab, ins, _ in bl:
            if IN[lab] != "unreached":
                transfer(IN[lab], ins, report, fn)
    return funcs, ndma, report


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--asm")
    p.add_argument("--define", action="append", default=[])
    a = p.parse_args()
    path = a.asm or compile_asm(a.define)
    funcs, ndma, report = scan(path)
    kern = [f for f in funcs if any(DMA.match(x) for x in funcs[f])]
    print(f"{path}: {len(funcs)} functions, {len(kern)} with LDS DMA ({ndma} DMA instructions)")
    for fn in kern:
        bad = [r for r in report if r[0] == fn]
        print(f"  {fn[:110]}: {'OK' if not bad else f'{len(bad)} uncovered LDS read(s)'}")
        for _, op, after in bad[:5]:
            print(f"      {op}  ({after} vector-memory ops behind the DMA on the worst path)")
    sys.exit(1 if report else 0)


if __name__ == "__main__":
    main()
