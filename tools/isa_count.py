#!/usr/bin/env python3
"""Static instruction counts per kernel of a hipcc --save-temps gfx950 .s file
(VALU, fp64 FMA, packed fp32 FMA, conversions, LDS, scalar loads, cache
maintenance): a quick check of what a source change did to a kernel.

    python tools/isa_count.py file.s [name-filter]
    python tools/isa_count.py --check-handoff file.s

--check-handoff (run by __graft_entry__.build()): the single-pass chain kernels
(k_chain_tile, k_chain_gct, k_chain_gen; not their rare-path repair kernels,
whose timing does not matter) must issue their SRC and pass-1 work
before the tile hand-off wait (csrc/chain_tile.hip, tile_cascade): no
v_pk_fma_f32 (the SRC's and pass 1's packed FMAs) after the poll loop's first
s_sleep in the listing, and pass 1's float64 change of basis (66 v_fma_f64)
ahead of it.  A compiler that sank them past the wait serialised the tiles of a
channel (10x slower); this turns the pin() guards
into a checked invariant.
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


def check_handoff(path):
    s = open(path).read()
    heads = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\w+):", s, re.M)]
    bad, seen = [], 0
    for i, (pos, name) in enumerate(heads):
        if not re.search(r"k_chain_(tile|gct|gen)", name) or "_repair" in name:
            continue
        seen += 1
        end = heads[i + 1][0] if i + 1 < len(heads) else len(s)
        lines = s[pos:end].split(".Lfunc_end")[0].split("\n")
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
    return seen, bad


if __name__ == "__main__":
    if sys.argv[1] == "--check-handoff":
        n, bad = check_handoff(sys.argv[2])
        if bad:
            print("hand-off ordering check FAILED:\n  " + "\n  ".join(bad))
            sys.exit(1)
        print(f"hand-off ordering check: {n} single-pass kernels issue SRC and pass 1 before the wait")
        sys.exit(0)
    for name, d in counts(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "").items():
        print(name[:70], " ".join(f"{k}={v}" for k, v in d.items()))
