#!/usr/bin/env python3
"""Like-for-like table of the reference's published grids from the
harness ports' outputs (profiles/r02_sweeps/*.txt): SpGEMM_alg_comparison (n in {512, 1024}
x density in {0.1, 0.5}, fp32, H2D inside the timed op, 100 runs) and the SpGEMM half of
SpGEMM_vs_SpMV (4 x 4 grid, scipy CPU vs GPU, A_csr @ B_csr).  The reference's numbers are
from different hardware (an NVIDIA GPU with cuSPARSE): context only."""
import re
import sys

REF_1A = {  # (n, rho, alg) -> (ms, dPeak) -- BASELINE.md 1a (figures/alg_comparison.png)
    (512, 0.1, 1): (0.8249, "36 MB"), (512, 0.1, 2): (0.8282, "18 MB"), (512, 0.1, 3): (1.7112, "20 MB"),
    (512, 0.5, 1): (3.8035, "776 MB"), (512, 0.5, 2): (4.8802, "370 MB"), (512, 0.5, 3): (7.2505, "318 MB"),
    (1024, 0.1, 1): (2.1494, "258 MB"), (1024, 0.1, 2): (2.4330, "174 MB"), (1024, 0.1, 3): (3.8103, "122 MB"),
    (1024, 0.5, 1): (67.0011, "6.03 GB"), (1024, 0.5, 2): (74.4531, "4.53 GB"), (1024, 0.5, 3): (100.9707, "2.44 GB"),
}
REF_1B = {  # (n, rho) -> (cpu ms, gpu ms) -- BASELINE.md 1b (figures/SPGEMM-gpu-speedup.png)
    (128, 0.01): (0.27, 0.48), (128, 0.05): (0.31, 0.48), (128, 0.1): (0.46, 0.50), (128, 0.5): (0.93, 0.62),
    (256, 0.01): (0.27, 0.49), (256, 0.05): (0.62, 0.50), (256, 0.1): (1.36, 0.61), (256, 0.5): (4.23, 0.83),
    (512, 0.01): (0.37, 0.48), (512, 0.05): (3.11, 0.66), (512, 0.1): (5.47, 0.82), (512, 0.5): (26.74, 3.67),
    (1024, 0.01): (0.99, 0.59), (1024, 0.05): (16.98, 1.10), (1024, 0.1): (24.94, 2.08), (1024, 0.5): (200.54, 66.80),
}


def alg_table(path):
    rows, cur = [], None
    for line in open(path):
        m = re.match(r"size = (\d+), density = ([\d.]+)", line)
        if m:
            cur = (int(m.group(1)), float(m.group(2)))
        m = re.match(r"A_csr @ B_csr \(alg=(\d)\)\s+([\d.]+)\s+(.+?B)\s+(.+?B)\s+([\d.]+)", line)
        if m and cur:
            rows.append((cur[0], cur[1], int(m.group(1)), float(m.group(2)), m.group(3).strip(),
                         m.group(4).strip(), float(m.group(5))))
    print("| n | density | alg | time ms (MI355X, H2D incl.) | dPeak VRAM | library peak | GFLOPS | reference ms | reference dPeak | time ratio ref/ours |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for n, d, a, t, dp, lp, gf in rows:
        rt, rdp = REF_1A.get((n, d, a), (None, "-"))
        print(f"| {n} | {d} | {a} | {t:.3f} | {dp} | {lp} | {gf:.1f} | {rt} | {rdp} | {rt / t:.1f}x |" if rt else
              f"| {n} | {d} | {a} | {t:.3f} | {dp} | {lp} | {gf:.1f} | - | - | - |")


def vs_table(path):
    cpu, gpu, cur, side = {}, {}, None, "cpu"
    for line in open(path):
        m = re.match(r">>> Running size = (\d+)\s+Running density = ([\d.]+)", line)
        if m:
            cur, side = (int(m.group(1)), float(m.group(2))), "cpu"
        if "=== Config (GPU" in line:
            side = "gpu"
        m = re.match(r"A_csr @ B_csr \(SpGEMM\)\s+([\d.]+)", line)
        if m and cur:
            (cpu if side == "cpu" else gpu)[cur] = float(m.group(1))
    print("| n | density | scipy CPU ms (GPU box host) | GPU ms (MI355X, H2D incl.) | speedup | reference CPU / GPU ms | reference speedup |")
    print("|---|---|---|---|---|---|---|")
    for key in sorted(REF_1B):
        if key in cpu and key in gpu:
            rc, rg = REF_1B[key]
            print(f"| {key[0]} | {key[1]} | {cpu[key]:.3f} | {gpu[key]:.3f} | {cpu[key] / gpu[key]:.2f}x | "
                  f"{rc} / {rg} | {rc / rg:.2f}x |")


if __name__ == "__main__":
    # usage: reference_grid.py [dir with r02_*.txt] | [alg_comparison.txt [spgemm_vs_spmv.txt]]
    arg = sys.argv[1] if len(sys.argv) > 1 else "profiles/r02_sweeps"
    if arg.endswith(".txt"):
        alg_file, vs_file = arg, (sys.argv[2] if len(sys.argv) > 2 else None)
    else:
        alg_file, vs_file = f"{arg}/r02_alg_comparison.txt", f"{arg}/r02_spgemm_vs_spmv.txt"
    print("### SpGEMM_alg_comparison grid (fp32, 100 runs, median; reference: BASELINE.md 1a, different hardware, context only)\n")
    alg_table(alg_file)
    if vs_file:
        print("\n### SpGEMM_vs_SpMV, SpGEMM half (A_csr @ B_csr; reference: BASELINE.md 1b, different hardware, context only)\n")
        vs_table(vs_file)
