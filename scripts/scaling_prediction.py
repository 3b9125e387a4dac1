#!/usr/bin/env python3
"""PREDICTED strong scaling of the headline (C2, 1920x1080x500) at N = 1/2/4/8 MI355X from one-GPU
measurements: every rank's rows rendered alone (scripts/gpu_shards.sh: bench.py --shard r/N, the
timed kernel's HIP-event time per step) plus a gather model.  Nothing here ran on more than one device.

  python scripts/scaling_prediction.py gpurun_out/shards06/shards.jsonl <full-frame ms> > profiles/r06_scaling_predicted.json

A step at N ranks (bench.py --gpus N) = the slowest rank's render + the nccl gather of the padded shards
to rank 0 + the de-interleave on rank 0.  The gather is modelled, not measured: rank 0 receives N-1 shards of
R x W x 12 B (R = ceil(H / N)), each over its own xGMI link of the fully connected 8-GPU node at
XGMI_GBS per direction (MI355X_MICROARCH.md: 7 links x ~153 GB/s bidirectional per GPU), concurrently,
plus GATHER_LAT_MS of collective latency; the de-interleave reads and writes the image once at COPY_GBS.
"""
import json
import sys

XGMI_GBS = 64.0       # per link and direction, sustained (half of the ~153 GB/s bidirectional figure, less overhead)
GATHER_LAT_MS = 0.03  # RCCL gather launch + handshake
COPY_GBS = 3000.0     # rank 0's permute-reshape copy of the image (device copy)
W, H = 1920, 1080

rows = [json.loads(line) for line in open(sys.argv[1]) if line.strip()]
full_ms = float(sys.argv[2])
out = {"workload": "random_spheres:1920x1080x500", "kind": "predicted (one-GPU shard renders + gather model)",
       "model": {"xgmi_gbs_per_link": XGMI_GBS, "gather_latency_ms": GATHER_LAT_MS, "copy_gbs": COPY_GBS},
       "librtx_sha256_16": sorted({r.get("librtx_sha256_16") for r in rows} - {None}), "n": {}}
out["n"]["1"] = {"max_rank_ms": full_ms, "gather_ms": 0.0, "step_ms": full_ms, "speedup": 1.0, "efficiency": 1.0}
for n in sorted({r["world"] for r in rows}):
    rk = sorted((r for r in rows if r["world"] == n), key=lambda r: r["rank"])
    assert [r["rank"] for r in rk] == list(range(n)), f"N={n}: ranks {[r['rank'] for r in rk]}"
    ms = [r["kernel_ms_avg"] or r["ms_per_step"] for r in rk]
    R = (H + n - 1) // n
    shard_mb = R * W * 12 / 1e6
    gather = GATHER_LAT_MS + shard_mb / XGMI_GBS  # the N-1 shards arrive concurrently, one link each
    gather += 2 * W * H * 12 / 1e6 / COPY_GBS     # de-interleave on rank 0
    step = max(ms) + gather
    out["n"][str(n)] = {"rank_ms": [round(v, 3) for v in ms], "max_rank_ms": round(max(ms), 3),
                        "mean_rank_ms": round(sum(ms) / n, 3), "imbalance": round(max(ms) / (sum(ms) / n), 4),
                        "shard_mb": round(shard_mb, 2), "gather_ms": round(gather, 3), "step_ms": round(step, 3),
                        "speedup": round(full_ms / step, 3), "efficiency": round(full_ms / step / n, 3)}
json.dump(out, sys.stdout, indent=1)
print()
