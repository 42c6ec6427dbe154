#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of tools/pmc.sh for one kernel.

Reads gpurun_out/pmc/p*/run_counter_collection.csv and writes a JSON summary
(per-launch means of every counter for the kernel) with the HBM traffic
estimate bench.py reports as roofline.traffic:

  traffic = 2 * FETCH_SIZE + WRITE_SIZE   (bytes per launch)

FETCH_SIZE / WRITE_SIZE are in KiB.  The factor 2 is the gfx950 correction of
MI355X_MICROARCH.md ("FETCH_SIZE reports exactly 1/2 of the bytes of a wide
coalesced streaming read"); tools/calib/fetch_calib.hip measured the same
0.5 for 2-, 4-, 8- and 16-byte reads and gathers of known distinct bytes
(profiles/r04b_fetch_calibration.json), so it applies to the warp's gathers.

usage: python tools/pmc_summary.py [pmc_dir] [kernel_substring] [out.json]
"""
import collections
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    kern = sys.argv[2] if len(sys.argv) > 2 else "render_fast"
    out = sys.argv[3] if len(sys.argv) > 3 else None
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    means = {k: sum(v) / len(v) for k, v in agg.items()}
    h = hashlib.sha256(open(os.path.join(ROOT, "gsky_amd", "libgskyhip.so"), "rb").read()).hexdigest()[:16]
    res = {"kernel_substring": kern, "counters_per_launch": means, "lib_sha16": h}
    m = means
    if "SQ_WAVE_CYCLES" in m and m.get("SQ_WAVE_CYCLES"):
        res["wait_any_frac"] = m.get("SQ_WAIT_ANY", 0) / m["SQ_WAVE_CYCLES"]
        res["valu_active_frac_of_wave_cycles"] = m.get("SQ_ACTIVE_INST_VALU", 0) / m["SQ_WAVE_CYCLES"]
    if "SQ_INSTS_VALU" in m and m.get("SQ_WAVES"):
        res["valu_insts_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
        res["vmem_rd_per_wave"] = m.get("SQ_INSTS_VMEM_RD", 0) / m["SQ_WAVES"]
    if "FETCH_SIZE" in means and "WRITE_SIZE" in means:
        fetch = means["FETCH_SIZE"] * 1024.0
        write = means["WRITE_SIZE"] * 1024.0
        res["fetch_bytes_raw"] = fetch
        res["write_bytes"] = write
        res["hbm_bytes_per_launch"] = 2.0 * fetch + write
        res["note"] = ("traffic = 2*FETCH_SIZE + WRITE_SIZE: FETCH_SIZE reports 0.5 of the distinct bytes for 2/4/8/16-B "
                       "reads and gathers on gfx950, WRITE_SIZE exact (profiles/r04b_fetch_calibration.json)")
    s = json.dumps(res, indent=1, sort_keys=True)
    if out:
        with open(out, "w") as fh:
            fh.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
