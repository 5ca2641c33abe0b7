"""Prints a per-kernel table (VGPRs, SGPRs, scratch, LDS, occupancy) from
hipcc -Rpass-analysis=kernel-resource-usage for the libdspcore sources."""
import re
import subprocess
import sys
import os

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dsp-audio-project_amd", "csrc")
files = sys.argv[1:] or ["src_poly.hip", "iir.hip", "fft.hip"]
for f in files:
    out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                          "-I../../include", "-I.", "-c", f, "-o", "/dev/null",
                          "-Rpass-analysis=kernel-resource-usage"] + (["-fno-slp-vectorize"] if f == "iir.hip" else []), cwd=CSRC,
                         capture_output=True, text=True).stderr
    cur = None
    rows = []
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
            name = re.sub(r"dsp::\(anonymous namespace\)::", "", name)
            name = re.sub(r"\(.*", "", name)
            cur = {"name": name}
            rows.append(cur)
            continue
        for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("sgpr", r"TotalSGPRs: (\d+)"),
                         ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, line)
            if m and cur is not None:
                cur[key] = int(m.group(1))
    for r in rows:
        print(f"{r.get('vgpr','?'):>4} vgpr {r.get('sgpr','?'):>4} sgpr {r.get('scratch','?'):>5} scr "
              f"{r.get('lds','?'):>6} lds occ {r.get('occ','?'):>2}  {r['name']}")
