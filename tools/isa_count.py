#!/usr/bin/env python3
"""Static instruction counts per kernel of a hipcc --save-temps gfx950 .s file
(VALU, fp64 FMA, packed fp32 FMA, conversions, LDS, scalar loads, cache
maintenance): a quick check of what a source change did to a kernel.

    python tools/isa_count.py file.s [name-filter]
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


if __name__ == "__main__":
    for name, d in counts(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "").items():
        print(name[:70], " ".join(f"{k}={v}" for k, v in d.items()))
