"""tools/pmc_parse.py, the summariser behind roofline.traffic and the PMC
figures DESIGN.md quotes: the HBM-bytes formula of MI355X_MICROARCH.md
((2 * FETCH_SIZE + WRITE_SIZE) KiB per launch on gfx950), the kernel naming
the bench's trace uses, and the derived clock / VALU-busy that are reported
only for dispatches long enough for GRBM_GUI_ACTIVE to mean the kernel (round
4's 5-8 GHz "clocks" of short dispatches), on synthetic rocprofv3 CSV passes."""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pmc_parse  # noqa: E402

CHAIN = "void dsp::(anonymous namespace)::k_chain_tile<dsp::(anonymous namespace)::TileGeo<3, 2, 41, 0>, true>(dsp::(anonymous namespace)::TileArgs)"  # noqa: E501
SPEC = "dsp::(anonymous namespace)::k_spec_wave12(dsp::(anonymous namespace)::FftArgs)"


def _pass(d, counters, durations_ns):
    """One rocprofv3 --pmc pass: counter_collection and kernel_trace CSVs."""
    os.makedirs(d)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        for i, (name, cname, v) in enumerate(counters):
            w.writerow([i, name, cname, v])
    with open(os.path.join(d, "run_kernel_trace.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for name, ns in durations_ns:
            w.writerow([name, 1000, 1000 + ns])


def test_short_names():
    assert pmc_parse.short(CHAIN) == "chain_tile"
    assert pmc_parse.short(SPEC) == "spectrum"
    assert pmc_parse.short("dsp::(anonymous namespace)::k_nf_list(dsp::NfArgs)") == "spectrum_nf"
    assert pmc_parse.short("void dsp::(anonymous namespace)::k_chain_gct_repair<160, 147, true>"
                           "(dsp::(anonymous namespace)::TileArgs)") == "chain_repair"
    assert pmc_parse.short("at::native::vectorized_elementwise_kernel<4>") is None


def test_traffic_clock_and_gating(tmp_path, capsys):
    root = str(tmp_path)
    # pass 1: fetch / write; pass 2: clock counters with the kernels' durations
    _pass(os.path.join(root, "p1"),
          [(CHAIN, "FETCH_SIZE", 1000.0), (CHAIN, "WRITE_SIZE", 500.0),
           (SPEC, "FETCH_SIZE", 10.0), (SPEC, "WRITE_SIZE", 4.0)],
          [(CHAIN, 5_000_000), (SPEC, 30_000)])
    # chain: 8 XCDs x 1.5 GHz x 5 ms of GRBM cycles; VALU quad-cycles for a
    # 0.9 share; spectrum: a 30 us dispatch whose GRBM window spans 6 GHz
    grbm = 8 * 1.5 * 5_000_000
    valu = 0.9 * (grbm / 8) * pmc_parse.N_SIMD / 4
    _pass(os.path.join(root, "p2"),
          [(CHAIN, "GRBM_GUI_ACTIVE", grbm), (CHAIN, "SQ_ACTIVE_INST_VALU", valu),
           (SPEC, "GRBM_GUI_ACTIVE", 8 * 6.0 * 30_000)],
          [(CHAIN, 5_000_000), (SPEC, 30_000)])
    out = pmc_parse.main(root)
    assert out["chain_tile"]["traffic_bytes"] == (2 * 1000 + 500) * 1024
    assert out["spectrum"]["traffic_bytes"] == (2 * 10 + 4) * 1024
    assert abs(out["chain_tile"]["clock_ghz"] - 1.5) < 1e-9
    assert abs(out["chain_tile"]["valu_busy_frac"] - 0.9) < 1e-9
    assert out["spectrum"]["clock_ghz"] == "n/a"
    assert out["spectrum"]["valu_busy_frac"] == "n/a"
    assert "n/a" in capsys.readouterr().out
