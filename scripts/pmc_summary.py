#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc runs (scripts/pmc_step.sh) per kernel: mean counter value per
dispatch, kernel time from the kernel trace of the same run, and derived rates:

* MFMA TF/s  = SQ_INSTS_MFMA x 32768 FLOP (v_mfma_f32_32x32x16_bf16; 16x16x32 is the same
  MAC count) / kernel time, and its share of the 2.5 PFLOP/s dense bf16 peak;
* MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) (rocprof's
  MfmaUtil; GRBM_GUI_ACTIVE is summed over the 8 XCDs);
* HBM GB/s   = (TCC_EA0_RDREQ + TCC_EA0_WRREQ) x 64 B / kernel time (lower bound: 128 B
  requests count once), share of 8 TB/s;
* L2 hit     = TCC_HIT / (TCC_HIT + TCC_MISS);
* LDS bank conflicts per LDS instruction, VALU instructions per MFMA.
"""
import collections
import csv
import glob
import os
import sys

PEAK_TF, PEAK_GBS = 2500.0, 8000.0


def main(root):
    cnt = collections.defaultdict(lambda: collections.defaultdict(list))
    tim = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "g*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            cnt[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in sorted(glob.glob(os.path.join(root, "g*", "**", "*kernel_trace.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            tim[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    rows = []
    for k, cs in cnt.items():
        ts = sorted(tim.get(k, []))
        if not ts:
            continue
        t = ts[len(ts) // 2]  # median dispatch time (counters serialise dispatches)
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        rows.append((sum(ts) / len(glob.glob(os.path.join(root, "g*"))), k, t, m))
    rows.sort(key=lambda r: -r[0])
    print(f"{'kernel':60s} {'us/disp':>8s} {'MFMA TF/s':>9s} {'%peak':>6s} {'MFMAbusy':>8s} {'HBM GB/s':>9s} "
          f"{'%HBM':>5s} {'L2hit':>6s} {'LDSconf/inst':>12s} {'VALU/MFMA':>9s}")
    for _, k, t, m in rows[:25]:
        mf = m.get("SQ_INSTS_MFMA", 0.0)
        tf = mf * 32768 / t / 1e12 if t > 0 else 0.0
        busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(1.0, m.get("GRBM_GUI_ACTIVE", 0.0) / 8 * 1024)
        hbm = (m.get("TCC_EA0_RDREQ_sum", 0.0) + m.get("TCC_EA0_WRREQ_sum", 0.0)) * 64 / t / 1e9 if t > 0 else 0.0
        hit = m.get("TCC_HIT_sum", 0.0) / max(1.0, m.get("TCC_HIT_sum", 0.0) + m.get("TCC_MISS_sum", 0.0))
        ldsc = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, m.get("SQ_INSTS_LDS", 0.0))
        vpm = m.get("SQ_INSTS_VALU", 0.0) / max(1.0, mf)
        name = k.replace("raft_amd::", "").replace("(anonymous namespace)::", "")[:60]
        print(f"{name:60s} {t * 1e6:8.1f} {tf:9.0f} {100 * tf / PEAK_TF:6.1f} {busy:8.2f} {hbm:9.0f} "
              f"{100 * hbm / PEAK_GBS:5.1f} {hit:6.2f} {ldsc:12.3f} {vpm:9.2f}")
    print("\nraw mean counters per dispatch (top 12 kernels):")
    for _, k, t, m in rows[:12]:
        print(k[:100])
        print("   " + ", ".join(f"{c}={v:.4g}" for c, v in sorted(m.items())))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_step")
