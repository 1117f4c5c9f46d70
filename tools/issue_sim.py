#!/usr/bin/env python3
"""In-order issue model of a kernel's steady-state loop (from hipcc -save-temps
assembly): each wave issues in order; an instruction waits for its sources
(VALU latency, DPP latency) and for the wave's issue interval.  Reports cycles
per loop iteration for one lone wave and the dependency stalls, so a schedule
can be judged without a GPU.  Costs are the tools/ubench_valu.hip numbers.

Usage: python tools/issue_sim.py file.s KERNEL_SYMBOL [--iters 4]
"""
import re
import sys

LONE_ISSUE = 4.75     # one wave: cycles between issues (ubench "1wave ILP8")
LAT = 9.7             # dependent VALU -> VALU (ubench "1wave chain")
LAT_DPP = 17.9        # a DPP consumer of a VALU result (ubench dpp chain)
LONE_ISSUE_DPP = 12.7  # one wave: cycles after a DPP move before its next issue


def regs(tok):
    tok = tok.strip().rstrip(",")
    m = re.match(r"([vs])\[(\d+):(\d+)\]", tok)
    if m:
        return [f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)]
    m = re.match(r"([vs])(\d+)$", tok)
    if m:
        return [tok]
    if tok in ("vcc", "exec"):
        return [tok]
    return []


def loops(path, sym):
    """Every innermost loop body (Loop Header .. first backward conditional branch)."""
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i] or
               l_is_end(lines[i], sym))
    body = lines[start:end]
    found = []
    for h in [i for i, l in enumerate(body) if "Loop Header" in l]:
        out = []
        for l in body[h + 1:]:
            s = l.strip()
            if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
                continue
            out.append(s)
            if s.startswith("s_cbranch"):
                break
        found.append(out)
    return found


def l_is_end(line, sym):
    return line.startswith(".Lfunc_end") and sym in line


def parse_loop(path, sym, want="v_pk_maximum3_f16", avoid=None):
    """The DP loop: the largest loop containing `want` (and not `avoid`)."""
    cands = [l for l in loops(path, sym) if any(want in i for i in l)
             and not (avoid and any(avoid in i for i in l))]
    return max(cands, key=len)


def simulate(instrs, iters):
    ready = {}
    t = 0.0
    gap = LONE_ISSUE
    per_iter = []
    stall = {}
    for it in range(iters):
        t0 = t
        for k, ins in enumerate(instrs):
            op = ins.split()[0]
            ops = ins[len(op):].split(";")[0]
            toks = [x for x in re.split(r"[ ,]+", ops) if x]
            if op.startswith("s_waitcnt") or op.startswith("s_cbranch") or op.startswith("s_"):
                t += 1.0
                continue
            dst = regs(toks[0]) if toks else []
            srcs = [r for tk in toks[1:] for r in regs(tk)]
            is_dpp = "_dpp" in op or "row_" in ins or "wave_shr" in ins
            start = t + (gap if k or it else 0)
            dep = max([ready.get(r, 0) for r in srcs] or [0])
            if is_dpp:
                dep = max([ready.get(r, 0) - LAT + LAT_DPP for r in srcs] or [0])
            issue = max(start, dep)
            if it == iters - 1 and issue > start:
                stall[k] = issue - start
            t = issue
            gap = LONE_ISSUE_DPP if is_dpp else LONE_ISSUE
            for r in dst:
                ready[r] = t + LAT
        per_iter.append(t - t0)
    return per_iter, stall


def main():
    path, sym = sys.argv[1], sys.argv[2]
    iters = int(sys.argv[sys.argv.index("--iters") + 1]) if "--iters" in sys.argv else 4
    want = sys.argv[sys.argv.index("--want") + 1] if "--want" in sys.argv else "v_pk_maximum3_f16"
    avoid = sys.argv[sys.argv.index("--avoid") + 1] if "--avoid" in sys.argv else None
    ins = parse_loop(path, sym, want, avoid)
    per, stall = simulate(ins, iters)
    nv = sum(1 for i in ins if i.startswith("v_"))
    print(f"instrs {len(ins)} (VALU {nv}); cycles/iter {per[-1]:.0f} "
          f"(no-stall {nv * LONE_ISSUE:.0f}); stall cycles {sum(stall.values()):.0f}")
    if "-v" in sys.argv:
        for k, i in enumerate(ins):
            print(f"{k:4d} {stall.get(k, 0):6.1f}  {i}")


if __name__ == "__main__":
    main()


FULL = ("v_xor_b32", "v_add_u32", "v_sub_u32", "v_subrev_u32", "v_max_u16", "v_min_u16", "v_sub_u16",
        "v_add_u16", "v_max_i16", "v_max_f16", "v_add_f16", "v_mov_b32", "v_and_b32", "v_or_b32",
        "v_not_b32", "v_cndmask_b32")


def cost(ins):
    op = ins.split()[0]
    if "_dpp" in op or "row_" in ins or "wave_shr" in ins:
        return 4.4
    if op.startswith("v_max3_u16") or op.startswith("v_max3_i16") or op.startswith("v_med3_u16"):
        return 8.1
    base = op.replace("_e32", "").replace("_e64", "").replace("_sdwa", "")
    if base in FULL and "_sdwa" not in op:
        return 2.2
    return 4.1


def simulate_simd(waves):
    """waves: list of (instrs, iterations).  Shared VALU, per-wave in-order issue."""
    state = []
    for ins, n in waves:
        pre = []
        for s in ins:
            op = s.split()[0]
            toks = [x for x in re.split(r"[ ,]+", s[len(op):].split(";")[0]) if x]
            salu = op.startswith("s_")
            dst = [] if salu else (regs(toks[0]) if toks else [])
            srcs = [] if salu else [r for tk in toks[1:] for r in regs(tk)]
            dpp = "_dpp" in op or "row_" in s or "wave_shr" in s
            pre.append((salu, dst, srcs, dpp, cost(s)))
        state.append({"ins": pre, "left": n * len(pre), "pc": 0, "t": 0.0, "ready": {}})
    valu_free = 0.0
    while any(w["left"] for w in state):
        best = None
        for w in state:
            if not w["left"]:
                continue
            salu, dst, srcs, dpp, c = w["ins"][w["pc"]]
            if salu:
                when = w["t"]
            else:
                dep = max([w["ready"].get(r, 0) + (LAT_DPP - LAT if dpp else 0) for r in srcs] or [0])
                when = max(w["t"], dep, valu_free)
            if best is None or when < best[0]:
                best = (when, w)
        when, w = best
        salu, dst, srcs, dpp, c = w["ins"][w["pc"]]
        if salu:
            w["t"] = when + 1.0
        else:
            valu_free = when + c
            w["t"] = when + (LONE_ISSUE_DPP if dpp else LONE_ISSUE)
            for r in dst:
                w["ready"][r] = when + LAT
        w["pc"] = (w["pc"] + 1) % len(w["ins"])
        w["left"] -= 1
    return max(w["t"] for w in state)
