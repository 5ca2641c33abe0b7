"""Summarises rocprofv3 --pmc CSV passes per kernel (mean over dispatches).

HBM traffic per launch (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads exactly half
the bytes of a 16-B-per-lane coalesced stream on gfx950, so
    traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes.
With --write WORKLOAD CHANNELS SOURCE it records the per-launch traffic in
pmc_traffic.json (repo root) under the bench workload name (config3, config4,
config5) for that batch; bench.py reports it as roofline.traffic when its own
batch matches."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

def short(name):
    """Bench-trace name of a libdspcore kernel from its demangled symbol."""
    if "_repair" in name:
        return "chain_repair"
    if "k_pcm_batch" in name or "k_scale_batch" in name:
        return "pcm_batch"
    if "k_chain_tile" in name or "k_chain_gen" in name or "k_chain_gct" in name:
        return "chain_tile"
    if "k_tile_prep" in name:
        return "chain_prep"
    if "k_src" in name:
        return "src_poly"
    if "k_spec_real" in name or "k_spec_stream" in name or "k_spec_wave" in name:
        return "spectrum"
    m = re.search(r"k_iir_wave<(\d+), (\d+)", name)
    if m:
        return {"2": "iir_xstate"}.get(m.group(2), "iir_fused")
    m = re.search(r"k_iir_pass<(\d+), (true|false)", name)
    if m:
        return "iir_apply" if m.group(2) == "true" else "iir_state"
    if "k_iir_carry" in name:
        return "iir_carry"
    if "k_iir_prep" in name:
        return "iir_prep"
    m = re.search(r"k_fft<(\d+), (\d+)", name)
    if m:
        return "spectrum" if m.group(2) == "2" else "fft"
    return None


def main(root, write=None):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                if k:
                    vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for k in sorted(vals):
        c = {n: sum(v) / len(v) for n, v in vals[k].items()}
        out[k] = c
        print(f"== {k}")
        for n in sorted(c):
            print(f"   {n:28s} {c[n]:.6g}")
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            t = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
            c["traffic_bytes"] = t
            print(f"   traffic (2*FETCH+WRITE)     {t / 1e9:.4f} GB per launch")
    if write:
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "pmc_traffic.json")
        data = {}
        if os.path.exists(path):
            with open(path) as fh:
                data = json.load(fh)
        wl, channels, source = write
        data[wl] = {"channels": int(channels), "source": source,
                    "per_launch": {k: round(c["traffic_bytes"]) for k, c in out.items()
                                   if "traffic_bytes" in c}}
        with open(path, "w") as fh:
            json.dump(data, fh, indent=1)
        print("wrote", path)
    return out


if __name__ == "__main__":
    w = None
    if "--write" in sys.argv:
        i = sys.argv.index("--write")
        w = tuple(sys.argv[i + 1:i + 4])
    main(sys.argv[1], w)
