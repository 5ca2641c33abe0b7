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
    if "k_nf_small" in name or "k_nf_list" in name or "k_nf_fix" in name:
        return "spectrum_nf"
    if "k_lfilter_nf" in name:
        return "lfilter_nf"
    if "k_pcm_batch" in name or "k_scale_batch" in name:
        return "pcm_batch"
    if "k_chain_tile_carry" in name or "k_tile_carry" in name:
        return "chain_tile_carry"
    if ("k_chain_pp3" in name or "k_chain_tile3" in name or "k_chain_gen3" in name or
            "k_chain_gct3" in name):
        return "chain_tile3"
    if ("k_chain_tile" in name or "k_chain_gen" in name or "k_chain_gc" in name or
            "k_chain_pp" in name):
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


N_SIMD = 1024      # MI355X: 256 CUs x 4 SIMDs
N_XCD = 8
# GRBM_GUI_ACTIVE counts the GPU's busy cycles over the whole counter window,
# which for a short dispatch includes the profiler's own time around it
# (round 4 printed 5-8 GHz "clocks" for 6-30 us kernels): the derived clock and
# VALU-busy share are reported only for dispatches of at least MIN_DERIVED_NS
# and only when the clock is physical (<= MAX_CLOCK_GHZ; MI355X peaks at 2.4).
MIN_DERIVED_NS = 50_000
MAX_CLOCK_GHZ = 2.5


def pass_durations(pass_dir):
    """Mean kernel duration (ns) per short name in one pass's kernel trace."""
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(pass_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                if k:
                    durs[k].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return {k: sum(v) / len(v) for k, v in durs.items()}


def main(root, write=None):
    vals = defaultdict(lambda: defaultdict(list))
    grbm_dur = defaultdict(list)   # kernel durations (ns) of the passes that count GRBM_GUI_ACTIVE
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        has_grbm = False
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                if k:
                    vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                    has_grbm = has_grbm or row["Counter_Name"] == "GRBM_GUI_ACTIVE"
        if has_grbm:
            for k, d in pass_durations(os.path.dirname(f)).items():
                grbm_dur[k].append(d)
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
        # effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration, MI355X_MICROARCH.md DVFS) and
        # the share of the kernel's cycles each SIMD issues VALU (SQ_ACTIVE_INST_VALU counts
        # quad-cycles: one per wave64 VALU instruction)
        if "GRBM_GUI_ACTIVE" in c and grbm_dur.get(k):
            cycles = c["GRBM_GUI_ACTIVE"] / N_XCD
            dur = sum(grbm_dur[k]) / len(grbm_dur[k])
            clock = cycles / dur
            if dur < MIN_DERIVED_NS or clock > MAX_CLOCK_GHZ:
                c["clock_ghz"] = c["valu_busy_frac"] = "n/a"
                print(f"   effective clock             n/a ({dur / 1e6:.4f} ms dispatch: "
                      f"GRBM_GUI_ACTIVE spans more than the kernel, {clock:.2f} GHz)")
            else:
                c["clock_ghz"] = clock
                print(f"   effective clock             {clock:.3f} GHz ({dur / 1e6:.4f} ms)")
                if "SQ_ACTIVE_INST_VALU" in c:
                    c["valu_busy_frac"] = c["SQ_ACTIVE_INST_VALU"] * 4 / N_SIMD / cycles
                    print(f"   VALU-busy share of cycles   {c['valu_busy_frac']:.3f}")
        if "SQ_INSTS_VALU" in c and c.get("SQ_WAVES"):
            c["valu_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
            print(f"   VALU per wave               {c['valu_per_wave']:.1f}")
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            c["lds_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
            print(f"   LDS bank-conflict share     {c['lds_conflict_frac']:.4f}")
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
                                   if "traffic_bytes" in c},
                    "derived": {k: {n: (round(c[n], 4) if isinstance(c[n], float) else c[n])
                                    for n in ("clock_ghz", "valu_busy_frac", "valu_per_wave",
                                              "lds_conflict_frac") if n in c}
                                for k, c in out.items()}}
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
