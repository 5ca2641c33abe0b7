#!/usr/bin/env python3
"""Static instruction counts per kernel of a hipcc --save-temps gfx950 .s file
(VALU, fp64 FMA, packed fp32 FMA, conversions, LDS, scalar loads, cache
maintenance): a quick check of what a source change did to a kernel.

    python tools/isa_count.py file.s [name-filter]
    python tools/isa_count.py --check-handoff file.s

--check-handoff (run by __graft_entry__.build()): the single-pass chain kernels
(k_chain_tile, k_chain_gct, k_chain_gen, k_chain_pp; not their rare-path repair kernels,
whose timing does not matter, nor the three-launch mode's k_chain_*3 kernels, which have no
hand-off) must issue their SRC and pass-1 work
before the tile hand-off wait (csrc/chain_tile.hip, tile_cascade): no
v_pk_fma_f32 (the SRC's and pass 1's packed FMAs) after the poll loop's first
s_sleep in the listing, and pass 1's float64 change of basis (66 v_fma_f64)
ahead of it.  A compiler that sank them past the wait serialised the tiles of a
channel (10x slower); this turns the pin() guards
into a checked invariant.

It also checks the counted wait of the early hand-off (round 4): a producer
raises its tile's flag (global_store_dword ... sc1) after `s_waitcnt vmcnt(N)`,
N > 0, which orders the flag after the tile's end-state stores
(global_store_dwordx2 ... sc1) only if at least N vector-memory instructions
are issued between those stores and the wait on EVERY path (vmcnt retires in
issue order on gfx950).  The check walks the listing's control flow (branch
targets and fall-through) from the state stores to each counted wait that
precedes a flag store and takes the fewest VMEM instructions on any path; a
compiler that merged, dropped or predicated away one of store_tile's y stores
fails the build.
"""
import re
import sys


def counts(path, filt=""):
    s = open(path).read()
    heads = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\w+):", s, re.M)]
    out = {}
    for i, (pos, name) in enumerate(heads):
        if filt not in name:
            continue
        end = heads[i + 1][0] if i + 1 < len(heads) else len(s)
        body = s[pos:end].split(".Lfunc_end")[0]

        def c(p):
            return len(re.findall(p, body, re.M))
        out[name] = dict(valu=c(r"^\s+v_"), fma_f64=c(r"^\s+v_fma_f64"), mul_f64=c(r"^\s+v_mul_f64"),
                         pk_fma=c(r"^\s+v_pk_fma_f32"), cvt=c(r"^\s+v_cvt_"), lds=c(r"^\s+ds_"),
                         s_load=c(r"^\s+s_load"), wbl2=c(r"buffer_wbl2"), inv=c(r"buffer_inv"))
    return out


VMEM = re.compile(r"^(buffer_|global_|flat_|scratch_)")
STATE_STORE = re.compile(r"^global_store_dwordx2\b.*\bsc1\b")
FLAG_STORE = re.compile(r"^global_store_dword\s.*\bsc1\b")
COUNTED_WAIT = re.compile(r"^s_waitcnt\b.*\bvmcnt\((\d+)\)")


def _program(lines):
    """Instructions (comments and directives dropped) and label -> index."""
    ins, labels = [], {}
    for raw in lines:
        t = raw.split(";")[0].strip()
        if not t or t.startswith("."):
            m = re.match(r"^(\.LBB\w+):", t)
            if m:
                labels[m.group(1)] = len(ins)
            continue
        if t.endswith(":"):
            continue
        ins.append(t)
    return ins, labels


def _min_vmem(ins, labels, starts, target):
    """Fewest VMEM instructions issued on any control-flow path from one of
    `starts` (exclusive) to `target` (exclusive): 0-1 breadth-first search over
    fall-through and branch edges."""
    from collections import deque
    INF = float("inf")
    dist = [INF] * (len(ins) + 1)
    dq = deque()
    for s0 in starts:
        if s0 + 1 < len(dist) and dist[s0 + 1] > 0:
            dist[s0 + 1] = 0
            dq.appendleft(s0 + 1)
    while dq:
        i = dq.popleft()
        if i == target or i >= len(ins):
            continue
        d = dist[i] + (1 if VMEM.match(ins[i]) else 0)
        op = ins[i].split()[0]
        succ = []
        if op == "s_endpgm":
            succ = []
        elif op == "s_branch":
            succ = [labels[ins[i].split()[1]]]
        elif op.startswith("s_cbranch"):
            succ = [i + 1, labels[ins[i].split()[1]]]
        else:
            succ = [i + 1]
        for j in succ:
            if d < dist[j]:
                dist[j] = d
                (dq.append if d > dist[i] else dq.appendleft)(j)
    return dist[target]


def check_counted_wait(ins, labels):
    """For every flag store that follows state stores: [(N, fewest VMEM
    instructions on any path from the state stores)] for each vmcnt(N > 0) wait
    between them (N = -1: the flag store has no vmcnt wait after the state
    stores at all)."""
    states = [i for i, t in enumerate(ins) if STATE_STORE.match(t)]
    out = []
    for f, t in enumerate(ins):
        if not FLAG_STORE.match(t) or not any(s < f for s in states):
            continue
        waits = [(i, int(COUNTED_WAIT.match(ins[i]).group(1))) for i in range(min(states), f)
                 if COUNTED_WAIT.match(ins[i])]
        if not waits:
            out.append((-1, 0))
        for w, n in waits:
            if n > 0:
                out.append((n, _min_vmem(ins, labels, [s for s in states if s < w], w)))
    return out


def check_handoff(path, text=None):
    s = open(path).read() if text is None else text
    heads = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\w+):", s, re.M)]
    bad, seen, report = [], 0, []
    for i, (pos, name) in enumerate(heads):
        # (k_chain_{pp,tile,gen,gct}3: launches 1 and 3 of the three-launch
        # mode, which wait for no other tile)
        if not re.search(r"k_chain_(tile|gct|gen|pp)", name) or "_repair" in name or \
                re.search(r"k_chain_(pp|tile|gen|gct)3", name):
            continue
        seen += 1
        end = heads[i + 1][0] if i + 1 < len(heads) else len(s)
        lines = s[pos:end].split(".Lfunc_end")[0].split("\n")
        prog, labels = _program(lines)
        for n, have in check_counted_wait(prog, labels):
            if n < 0:
                bad.append(f"{name}: a tile flag store with no vmcnt wait after the state stores")
                continue
            report.append(f"{name[:60]}: vmcnt({n}) after >= {have} VMEM on every path")
            if have < n:
                bad.append(f"{name}: counted hand-off wait vmcnt({n}) but only {have} vector-memory "
                           "instructions after the state stores on some path")
        ins = [l.strip() for l in lines]
        sleeps = [n for n, l in enumerate(ins) if l.startswith("s_sleep")]
        if not sleeps:
            bad.append(f"{name}: no hand-off poll loop (s_sleep) found")
            continue
        w = sleeps[0]
        pk_after = sum(1 for l in ins[w:] if l.startswith("v_pk_fma_f32"))
        f64_before = sum(1 for l in ins[:w] if l.startswith(("v_fma_f64", "v_fmac_f64")))
        if pk_after:
            bad.append(f"{name}: {pk_after} v_pk_fma_f32 after the hand-off wait")
        if f64_before < 66:
            bad.append(f"{name}: only {f64_before} v_fma_f64 before the hand-off wait (< 66)")
    if not seen:
        bad.append("no single-pass chain kernel in " + path)
    return seen, bad, report


if __name__ == "__main__":
    if sys.argv[1] == "--check-handoff":
        n, bad, report = check_handoff(sys.argv[2])
        for r in report:
            print("  " + r)
        if bad:
            print("hand-off ordering check FAILED:\n  " + "\n  ".join(bad))
            sys.exit(1)
        print(f"hand-off ordering check: {n} single-pass kernels issue SRC and pass 1 before the "
              f"wait; {len(report)} counted flag waits covered by their y stores")
        sys.exit(0)
    for name, d in counts(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "").items():
        print(name[:70], " ".join(f"{k}={v}" for k, v in d.items()))
