"""Per-kernel resource usage (VGPRs, AGPRs, scratch, LDS, occupancy) of one HIP source, from
the compiler's kernel-resource-usage remarks: python scripts/kernel_resources.py conv_igemm.hip
[--filter fwd6] [--scratch-only]."""
import argparse
import re
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from raft_ros_amd.csrc import build as b  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("source")
    ap.add_argument("--filter", default="")
    ap.add_argument("--scratch-only", action="store_true")
    args = ap.parse_args()
    flags, _ = b._common_flags()
    src = Path(args.source)
    if not src.exists():
        src = b.CSRC / args.source
    cmd = [b._hipcc(), "--offload-arch=gfx950", "--cuda-device-only", *flags, "-c", str(src), "-o", "/tmp/kr.o",
           "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        print(r.stderr[-4000:])
        sys.exit(r.returncode)
    rows, cur = [], None
    keys = {"VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch", "Occupancy [waves/SIMD]": "occ",
            "LDS Size [bytes/block]": "lds"}
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        for k, v in keys.items():
            m = re.search(re.escape(k) + r": (\d+)", line)
            if m and cur is not None:
                cur[v] = int(m.group(1))
    for row in rows:
        if args.filter not in row["name"]:
            continue
        if args.scratch_only and not row.get("scratch"):
            continue
        print(f"vgpr={row.get('vgpr', 0):3d} agpr={row.get('agpr', 0):3d} scratch={row.get('scratch', 0):4d} "
              f"lds={row.get('lds', 0):6d} occ={row.get('occ', 0)}  {row['name'][:120]}")


if __name__ == "__main__":
    main()
