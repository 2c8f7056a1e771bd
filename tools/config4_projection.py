"""configs[4]'s tree phase (n = 1e6 taxa, float LT, world 8), projected from
measured per-join device costs.  No 8-GPU node has been
available to this engine, so RCCL at world > 1 is unmeasured; its latency
and ring bandwidth are the model's parameters, stated in the output.

Inputs (measured on one MI355X, round 6):
  profiles/r06_shard_cost.jsonl  the sharded DNJ kernels at world 1 on
      configs[3]'s 200k float matrix: us per join by kernel class, engine
      cells per join (first 2000 / 20000 joins);
  profiles/r05_config4_rank.jsonl  one configs[4] rank's dist into its
      250 GB shard (6.40 s).
Model, per join at matrix size m (m = n .. 3), world W:
  chain(m)  = plan + pick/join + requeue: latency chains of a few dependent
              round trips whose grids grow with m / W; taken as their 200k,
              world-1 cost (an upper bound for a rank's 125k rows at 1e6);
  scan(m)   = the 200k scan's us per join x (m / 200k) / W: the rescans are
              a latency chain too, the bounded cells per row grow with m and
              a rank holds 1 / W of the rows;
  coll(m)   = 2 x RCCL latency + the allreduce ring bytes 2 (W-1)/W x 3 s m
              over the ring bandwidth + the record allgather (W-1)/W x
              W x (m / W) 13 B over the same.
    python tools/config4_projection.py [latency_us] [ring_GBps] > profiles/r06_config4_projection.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    lat_us = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    ring = float(sys.argv[2]) if len(sys.argv) > 2 else 300.0   # GB/s per rank into the ring (xGMI, 8 GPUs)
    rows = [json.loads(x) for x in open(os.path.join(ROOT, "profiles", "r06_shard_cost.jsonl"))]
    ref = max(rows, key=lambda r: r["joins"])
    per = ref["device_us_per_join"]
    chain = per["dnj_find"] + per["update"] + per["dnj_requeue"]
    scan200 = per["dnj_scan"]
    rank = json.loads(open(os.path.join(ROOT, "profiles", "r05_config4_rank.jsonl")).readline())
    n, W, s, m0 = 1_000_000, 8, 4, 200_000
    # sum over the joins (m = n .. 3) in closed form
    sum_m = (n * (n + 1) / 2) - 3.0
    joins = n - 2
    t_chain = joins * chain * 1e-6
    t_scan = scan200 * 1e-6 / W / m0 * sum_m
    t_lat = joins * 2 * lat_us * 1e-6
    bytes_ar = 2 * (W - 1) / W * 3 * s * sum_m
    bytes_ag = (W - 1) / W * 13 * sum_m
    t_bw = (bytes_ar + bytes_ag) / (ring * 1e9)
    tree_s = t_chain + t_scan + t_lat + t_bw
    # algorithmic HBM bytes of the tree phase over all ranks: the scans' cells (4 B) at the 200k engine rate of
    # cells per join scaled by (m / 200k)^2, plus ~ (4 s + 40) m of vectors and line updates per join
    cells = ref["engine_cells_per_join"] / m0 ** 2 * (n ** 3 / 3.0)
    algo_bytes = 4.0 * cells + (4 * s + 40) * sum_m
    out = {
        "what": "configs[4] tree phase (n = 1e6, float, world 8) projected from measured per-join parts; RCCL at "
                "world > 1 not measured on this pool (model parameters below)",
        "inputs": {"shard_cost": {k: ref[k] for k in ("n", "joins", "device_us_per_join", "engine_cells_per_join")},
                   "config4_rank_dist_s": rank["dist_s"]},
        "model": {"chain_us_per_join": round(chain, 2), "scan_us_per_join_at_200k_world1": scan200,
                  "rccl_latency_us": lat_us, "ring_GBps": ring},
        "tree_phase_s": {"kernel_chain": round(t_chain, 1), "scan": round(t_scan, 1),
                         "collective_latency": round(t_lat, 1), "collective_bytes": round(t_bw, 1),
                         "total": round(tree_s, 1)},
        "dist_phase_s": rank["dist_s"],
        "end_to_end_s": round(tree_s + rank["dist_s"], 1),
        "tree_phase_aggregate_hbm_fraction": round(algo_bytes / tree_s / (8.0e12 * W), 5),
        "reading": "the tree phase is a chain of ~1e6 dependent joins, each a few latency-bound kernels and two "
                   "collectives: its bytes are far below 30% of the aggregate HBM bandwidth whatever the world "
                   "size; the dist phase is MFMA-bound (0.45-0.57 of the fp4 dense peak per GPU)"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
