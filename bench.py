"""Benchmark: flow-check decisions/s on BASELINE.json's headline workload.

Workload (N=1): config 3 — 10M resources, Zipf(1.1) traffic, mixed QPS /
THREAD / WarmUp / RateLimiter rules, 2^27 events per batch (entries + exits),
consecutive batches 4 s of trace time apart.  A step = one sf_submit of one
batch whose inputs are already resident in HBM.  For N>1 each rank owns the
resources ``res % N == rank`` (hash sharding, no data-path collective) and
decides its own 2^27-event batch: weak scaling.

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement" for the byte
model behind ``roofline`` and for the cpu_baseline sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from sentinel_amd import abi, engine, trace  # noqa: E402

engine.lib()   # the HIP runtime of /opt/rocm is loaded before anything else

METRIC = "flow-check decisions/sec (node) + % HBM roofline, 10M resources, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
DURATION_MS = 4000             # trace time per batch


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--resources", type=int, default=10_000_000)
    ap.add_argument("--events", type=int, default=1 << 27)
    ap.add_argument("--no-cpu", action="store_true", help="skip the whole-batch oracle replay (parity + cpu_baseline)")
    ap.add_argument("--no-metric-log", action="store_true")
    ap.add_argument("--no-degrade", action="store_true")
    ap.add_argument("--no-legs", action="store_true", help="skip the config2 / config4 / config5 / end-to-end legs")
    ap.add_argument("--legs", default="", help="comma-separated subset of the legs to run (default: all)")
    ap.add_argument("--predict-ranks", type=int, default=0,
                    help="predict the N-GPU run on this one GPU: build the node-wide N-component trace on the host, "
                         "time the shard of the rank holding the Zipf head and of the lightest rank (one JSON line)")
    ap.add_argument("--origin-variants", default="no_origin_rules,other_rules_1pct",
                    help="config3_origin leg: the variants to run")
    ap.add_argument("--placement", type=int, default=16384,
                    help="N > 1: move the top-K resources (by the previous batch's counts) across the ranks, LPT "
                         "greedy (sentinel_amd/placement.py); 0 = every resource at res % N")
    ap.add_argument("--no-system-leg", action="store_true", help="N > 1: skip the RCCL SystemRule exchange leg")
    ap.add_argument("--heavy-min", type=int, default=0,
                    help="segments of more events than this go to the heavy kernels (0: the engine default, 512)")
    args = ap.parse_args()
    if args.predict_ranks > 1:
        predict_ranks(args)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)              # gloo prints its connection banner on stdout: keep stdout to the one JSON line
        try:
            dist.init_process_group("gloo")
        finally:
            os.dup2(saved, 1)
            os.close(saved)
    assert world == args.gpus or world == 1, "launch N>1 with torch.distributed.run"

    R_total = args.resources
    t0 = time.time()
    # the node-wide trace: N = 1 is config 3's batch; N > 1 superposes N
    # config-3 traces over all 10M resources (component c = seed 3 + c, built
    # by rank c) and shards the result, rank r keeping the resources the
    # placement gives it (the top-K by count spread LPT-greedy, the rest at
    # res % N; sentinel_amd/placement.py), renamed to their engine ids
    hb, pl = node_trace(R_total, args.events, world, rank, dist, args.placement)
    # rules of the whole node (config 3's table over the 10M resources), this
    # rank's shard, by engine id; per engine row (id // N) for the roofline model
    grade_all, beh_all, count_all = trace.mixed_rule_table(R_total, seed=3)
    if pl is None:
        mine_res = np.arange(rank, R_total, world, dtype=np.int64)
        mine_eid = mine_res
        R_local = (R_total - rank + world - 1) // world
    else:
        mine_res = np.nonzero(pl.owner(np.arange(R_total)) == rank)[0]
        mine_eid = pl.engine_id(mine_res)
        R_local = pl.local_rows()
    rules = abi.flow_rules_np(mine_eid.astype(np.uint32), grade_all[mine_res], count_all[mine_res], beh_all[mine_res])
    grade = np.zeros(R_local, np.int32)
    beh = np.zeros(R_local, np.int32)
    grade[mine_eid // world] = grade_all[mine_res]
    beh[mine_eid // world] = beh_all[mine_res]
    res_of_eid = None
    if pl is not None:
        res_of_eid = np.full(pl.R_pad + world * pl.extra, -1, np.int64)
        res_of_eid[pl.eid] = np.arange(R_total)
    del grade_all, beh_all, count_all, mine_res, mine_eid
    n_entry = int(((hb.flags & abi.EV_EXIT) == 0).sum())
    n_exit = hb.n - n_entry
    log(f"[rank {rank}] trace {hb.n} events ({n_entry} entries) over {R_local} resources in {time.time()-t0:.1f}s")

    cfg = abi.default_config(max_resources=R_local, max_batch=hb.n, shard_count=world, shard_index=rank,
                             device=local, heavy_min_events=args.heavy_min)
    eng = engine.FlowEngine(cfg)
    eng.load_flow_rules(rules)
    steps = args.warmup + args.steps
    # the batch resident in HBM once per step: timestamps shifted so that
    # consecutive batches continue the same trace (every other array shared)
    base = engine.DeviceBatch(eng, hb)
    batches = [base] + [engine.DeviceBatch.with_ts(eng, base, hb.ts_ms + k * DURATION_MS) for k in range(1, steps)]
    out = engine.DeviceVerdicts(eng, hb.n, with_wait=True, with_rule=False)
    out0 = engine.DeviceVerdicts(eng, hb.n, with_wait=True, with_rule=True)
    log(f"[rank {rank}] staged {steps} batches in HBM, t={time.time()-t0:.1f}s")

    # batches are enqueued (sf_submit_async): the engine sorts batch k+1 on
    # its sort stream while it decides batch k; decisions stay in batch order.
    # Batch 0 (fresh engine) keeps its verdicts for the whole-batch parity check.
    for k in range(args.warmup):
        eng.submit_device_async(batches[k], out0 if k == 0 else out)
    eng.sync()
    eng.set_timing(True)
    if dist:
        dist.barrier()
    eng.sync()
    start = time.perf_counter()
    for k in range(args.warmup, steps):
        eng.submit_device_async(batches[k], out)
    eng.sync()
    elapsed = time.perf_counter() - start
    if dist:
        dist.barrier()
    st = eng.stats()
    status = out.status.numpy()
    n_pass = int(np.isin(status, abi.PASSED).sum())
    wait = out.wait_ms.numpy()
    e_wait = int((wait > 0).sum())
    n_seg = int(st.n_segments)

    times = np.array([elapsed], np.float64)
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        times[0] = t.item()
        tot = torch.tensor([n_entry * args.steps], dtype=torch.float64)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        total_decisions = tot.item()
    else:
        total_decisions = n_entry * args.steps
    wall = times[0]
    value = total_decisions / wall
    per_rank = None
    if dist:
        box = [None] * world
        dist.all_gather_object(box, (int(hb.n), n_entry, round(elapsed / args.steps * 1e3, 3)))
        per_rank = {"events": [b[0] for b in box], "entries": [b[1] for b in box],
                    "ms_per_step": [b[2] for b in box],
                    "max_over_min_ms": round(max(b[2] for b in box) / max(1e-9, min(b[2] for b in box)), 3),
                    "max_over_mean_events": round(max(b[0] for b in box) / (sum(b[0] for b in box) / world), 3)}

    # roofline of the dominant decision kernel: SURVEY.md §8(d) byte model,
    # B = 25 E + 4 E_wait + 12 E_exit + 528 R_touched, restricted to the
    # segments (resources) that kernel decides.  Resources with more than
    # heavy_min events in the batch go to k_heavy_decide, the rest to
    # k_decide_light (sf_kernels.hip: k_classify).
    # k_classify routes segments of more than heavy_min events to the heavy
    # kernels: THREAD-grade and RateLimiter ones to k_heavy_stream, the rest
    # to k_heavy_decide.
    heavy_min = args.heavy_min or 512
    local = hb.res_id // world if world > 1 else hb.res_id
    per_res = np.bincount(local, minlength=R_local)
    is_heavy_res = per_res > heavy_min
    is_stream_rule = (grade == abi.GRADE_THREAD) | (beh == abi.BEHAVIOR_RATE_LIMITER)
    res_cls = np.where(~is_heavy_res, 0, np.where(is_stream_rule, 2, 1))
    ev_cls = res_cls[local]
    is_exit = (hb.flags & abi.EV_EXIT) != 0
    waited = wait > 0

    def alg_bytes(cls):
        sel = ev_cls == cls
        n_res = int(((per_res > 0) & (res_cls == cls)).sum())
        return int(25 * sel.sum() + 4 * (waited & sel).sum() + 12 * (is_exit & sel).sum() + 528 * n_res)

    n_heavy_res = int(is_heavy_res.sum())
    b_alg = 25 * hb.n + 4 * e_wait + 12 * n_exit + 528 * n_seg
    k = args.steps
    # single kernels timed live with HIP events on their own stream; the light
    # lanes are four kernels in a row on stream C (one event span), reported
    # beside the dominant kernel as "light_phase", not compared with it
    kern = {"k_heavy_decide": (st.heavy_decide_ms / k, alg_bytes(1)),
            "k_heavy_stream": (st.stream_ms / k, alg_bytes(2))}
    name = max(kern, key=lambda x: kern[x][0])
    ms, bytes_k = kern[name]
    achieved = bytes_k / (ms / 1e3) / 1e9
    # HBM bytes per launch from the committed rocprofv3 PMC passes of this
    # same command (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE)
    traffic, traffic_src = None, None
    light_names = ("k_decide_light", "k_decide_light_qps", "k_decide_short_qps", "k_decide_short")
    light_traffic = {}
    import glob
    # the latest round's profile of the final tree (r??_config3_summary_final.json),
    # else that round's plain summary
    profs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_config3_summary*.json")),
                   key=lambda p: (os.path.basename(p)[:3], p.endswith("_final.json")))
    prof = profs[-1] if profs else ""
    if prof:
        with open(prof) as fh:
            for kr in json.load(fh).get("kernels", []):
                kn = kr["kernel"].split("<")[0]
                if kr.get("hbm_bytes_per_launch") is None:
                    continue
                if kn == name:
                    traffic, traffic_src = int(kr["hbm_bytes_per_launch"]), os.path.relpath(prof, ROOT)
                if kn in light_names:
                    light_traffic[kn] = int(kr["hbm_bytes_per_launch"])
    light_ms, light_bytes = st.light_ms / k, alg_bytes(0)
    light_phase = {"kernels": list(light_names), "ms": round(light_ms, 4), "alg_bytes": light_bytes,
                   "achieved": round(light_bytes / (light_ms / 1e3) / 1e9, 2),
                   "frac": round(light_bytes / (light_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 5),
                   "traffic": sum(light_traffic.values()) if len(light_traffic) == len(light_names) else None}
    roofline = {"bound": "hbm", "kernel": name,
                "note": "achieved/frac: the dominant kernel's share of the byte model over its HIP-event time -- a "
                        "latency figure for a serial-chain kernel (k_heavy_stream reads pre-digested records); "
                        "pipeline.frac is the whole step's bytes over its wall time",
                "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "traffic_source": traffic_src,
                "alg_bytes_per_launch": bytes_k, "avg_launch_ms": round(ms, 4),
                "light_phase": light_phase,
                "pipeline": {"alg_bytes_per_step": b_alg,
                             "achieved_GBs": round(b_alg / (wall / k) / 1e9, 2),
                             "frac": round(b_alg / (wall / k) / 1e9 / HBM_PEAK_GBS, 5),
                             "heavy_segments": n_heavy_res},
                "kernels_ms": {"sort+segments+classify": round(st.sort_ms / k, 3),
                               "classify": round(st.classify_ms / k, 3),
                               "decide(join)": round(st.decide_ms / k, 3),
                               "k_decide_light": round(st.light_ms / k, 3),
                               "k_heavy_decide": round(st.heavy_decide_ms / k, 3),
                               "k_heavy_stream": round(st.stream_ms / k, 3),
                               "k_heavy_fill": round(st.heavy_fill_ms / k, 3),
                               "scatter": round(st.scatter_ms / k, 3)}}

    # (first after the timed region: the metrics.log leg below rolls every
    # node's current minute bucket, as StatisticNode.metrics() does)
    # whole-batch parity: batch 0 from a fresh engine vs the one-core oracle
    # replay of the same batch (that replay, timed, is the one-core CPU
    # baseline), then the steady state: the resource-sharded oracle replays
    # every batch of the run (warmup + timed, the first one timed as the
    # multi-core CPU baseline) and the last timed batch's verdicts, a sample of
    # nodes, their controller state and ENTRY_NODE are compared with the GPU's
    # the end-to-end form first, while the process's host memory is as the
    # service would have it at start-up: run after the CPU baseline's
    # multi-GB oracle replay its H2D period was 35 ms instead of 25 ms
    # (DESIGN.md "Round 4"); parity is against the headline run's verdicts
    legs = {}
    run_legs = rank == 0 and world == 1 and not args.no_legs
    want = (lambda nm: not args.legs or nm in args.legs.split(","))
    if run_legs:
        g0 = (out0.status.numpy(), out0.wait_ms.numpy(), out0.rule_idx.numpy())
        glast = (out.status.numpy(), out.wait_ms.numpy())
        if want("e2e_pinned"):
            try:
                t_leg = time.perf_counter()
                log("[leg e2e_pinned] ...")
                legs["e2e_pinned"] = e2e_leg(hb, rules, R_local, steps, g0, glast)
                log(f"[leg e2e_pinned] {time.perf_counter() - t_leg:.1f}s")
            except Exception as ex:  # pragma: no cover - reported, not fatal for the decision bench
                legs["e2e_pinned"] = {"error": str(ex)[:300]}

    cpu, parity = None, None
    if rank == 0 and world == 1 and not args.no_cpu and args.warmup > 0:
        cpu, parity = oracle_leg(rules, hb, R_local, out0, out, eng, steps, per_res)

    # node-wide ENTRY_NODE over the shards: RCCL all-reduce (off the decision
    # path, after the timed region)
    aggregate = None
    try:
        from sentinel_amd import dist as sdist
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)              # RCCL prints a version banner on stdout: keep stdout to the one JSON line
        try:
            if dist:
                sdist.rccl_join(eng)
            else:
                eng.comm_init(1, 0, engine.comm_unique_id())
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        eng.sync()
        t_ag = time.perf_counter()
        node = eng.entry_node_allreduce()
        aggregate = {"what": "ENTRY_NODE all-reduce (MAX window, SUM counters, MIN minRt)", "backend": "rccl",
                     "ranks": world, "ms": round((time.perf_counter() - t_ag) * 1e3, 3),
                     "node_threads": int(node.cur_thread_num)}
    except Exception as ex:  # pragma: no cover - reported, not fatal for the decision bench
        aggregate = {"error": str(ex)[:200]}

    # metrics.log leg (off the decision path): one MetricTimerListener.run
    # over this shard, after a drain fetch, so it covers one second of rows as
    # the reference's 1 s timer does (sf_metric_log)
    metric_log = None
    if not args.no_metric_log:
        try:
            metric_log = metric_log_leg(eng, hb, R_total, R_local, world, rank, steps, res_of_eid)
        except Exception as ex:  # pragma: no cover - reported, not fatal for the decision bench
            metric_log = {"error": str(ex)[:200]}

    # DegradeSlot leg (tools/degrade_bench.py has the full
    # version with the whole-batch oracle check): its own 1M-resource engine
    degrade = None
    if rank == 0 and world == 1 and not args.no_degrade:
        try:
            degrade = degrade_leg()
        except Exception as ex:  # pragma: no cover - reported, not fatal for the decision bench
            degrade = {"error": str(ex)[:200]}

    # the other BASELINE configs and the end-to-end form (rank 0, N=1 only;
    # after the timed region, each on its own engine except e2e)
    if run_legs:
        # the headline engine is released so that each leg has the device to itself
        for b in batches:
            b.free()
        batches = []
        base = None
        out0.free(); out.free()
        eng.close()
        c3_ms = wall / args.steps * 1e3
        for nm, fn in (# (4 batches: the oracle replays every batch of both variants,
                       # profiles/r04_config3_origin_parity.json holds a 7-batch run)
                       ("config3_origin", lambda: config3_origin_leg(hb, rules, R_local, c3_ms, steps=3, warmup=1,
                                                                       parity=not args.no_cpu,
                                                                       variants=args.origin_variants.split(","))),
                       ("config2", config2_leg), ("config4", config4_leg), ("config5", config5_leg)):
            if not want(nm):
                continue
            try:
                t_leg = time.perf_counter()
                log(f"[leg {nm}] ...")
                legs[nm] = fn()
                log(f"[leg {nm}] {time.perf_counter() - t_leg:.1f}s")
            except Exception as ex:  # pragma: no cover - reported, not fatal for the decision bench
                legs[nm] = {"error": str(ex)[:300]}

    # SystemRules on the sharded node (N > 1): config 4's shape decided through
    # the per-window exchange over RCCL (sf_submit_node)
    system_exchange = None
    if dist and not args.no_system_leg:
        try:
            system_exchange = system_exchange_leg(world, rank, int(os.environ.get("LOCAL_RANK", "0")), dist)
        except Exception as ex:  # pragma: no cover - reported, not fatal for the decision bench
            system_exchange = {"error": str(ex)[:300]}

    if rank == 0:
        line = {"metric": METRIC, "value": round(value, 1), "unit": "decisions/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
                "data": "synthetic",
                "config": {"workload": "config3: 10M resources Zipf(1.1), 60% QPS / 10% THREAD / 15% WarmUp / "
                                       "15% RateLimiter, acquireCount 1 (90%) or 2-5, RT~Exp(20ms) exits",
                           "resources": R_total, "events_per_batch_per_gpu": hb.n, "entries_per_batch_per_gpu": n_entry,
                           "resources_touched": n_seg, "pass_fraction": round(n_pass / max(1, n_entry), 4),
                           "parallelism": f"resource-sharded x{world}",
                           "placement": None if pl is None else
                           {"what": "top-K resources by count spread LPT-greedy over the ranks, the rest at res % N "
                                    "(counts of the previous batch: the bench's batches repeat one trace shifted "
                                    "in time)", "K": int(pl.moved.size), "engine_rows_per_rank": R_local},
                           "trace": "one node-wide trace: N config-3 batches of 2^27 events over all 10M resources "
                                    "(seeds 3..3+N-1, the same 4 s) superposed, rank r deciding res % N == r"
                                    if world > 1 else "config-3 batch, seed 3", "per_rank": per_rank},
                "roofline": roofline, "cpu_baseline": cpu, "parity": parity, "aggregate": aggregate,
                "metric_log": metric_log, "degrade": degrade, "system_exchange": system_exchange, **legs}
        print(json.dumps(line), flush=True)
    for b in batches[1:]:
        b.free()
    if base is not None:
        base.free()
    if dist:
        dist.destroy_process_group()


def node_trace(R_total, n, world, rank, dist, placement_k=0):
    """This rank's shard of one node-wide trace, and the placement.  Component
    c (built by rank c) is a config-3 batch of n events over all R_total
    resources (seed 3 + c, the same 4 s of trace time); the node's trace is
    the superposition of the N components (N times the traffic of one),
    merged in time order (events of one millisecond in component order), and
    sharded: by default rank r keeps the events of res % N == r, so the rank
    holding the Zipf head gets more events than the others; with placement_k
    the top-K resources by the node's counts (all-reduced over the ranks) are
    spread LPT-greedy (sentinel_amd/placement.py) and every event carries its
    resource's engine id.  Exits stay with their entries (same resource).
    The components' parts travel between ranks by all_to_all over the host
    process group."""
    comp = trace.mixed_zipf(R_total, n, duration_ms=DURATION_MS, seed=3 + rank)
    if world == 1:
        return comp, None
    import torch
    pl = None
    if placement_k:
        from sentinel_amd.placement import Placement
        cnt_t = torch.from_numpy(np.bincount(comp.res_id, minlength=R_total).astype(np.int64))
        dist.all_reduce(cnt_t)
        pl = Placement.balanced(cnt_t.numpy(), world, placement_k)
        del cnt_t
        comp.res_id = pl.engine_id(comp.res_id).astype(np.uint32)
    dest = (comp.res_id % world).astype(np.uint8)
    order = np.argsort(dest, kind="stable")
    send = np.bincount(dest, minlength=world).astype(np.int64)
    pos = np.empty(comp.n, np.int64)                       # index of each event inside its destination part
    starts = np.concatenate([[0], np.cumsum(send)])
    for d in range(world):
        idx = order[starts[d]:starts[d + 1]]
        pos[idx] = np.arange(idx.size)
    eref = np.where(comp.entry_ref >= 0, pos[np.clip(comp.entry_ref, 0, None)], -1)
    recv = torch.empty(world, dtype=torch.int64)
    dist.all_to_all_single(recv, torch.from_numpy(send))
    recv = recv.numpy()
    ss, rs = [int(x) for x in send], [int(x) for x in recv]

    def a2a(arr, dtype):
        x = torch.from_numpy(np.ascontiguousarray(arr[order]).astype(dtype, copy=False))
        y = torch.empty(sum(rs), dtype=x.dtype)
        dist.all_to_all_single(y, x, output_split_sizes=rs, input_split_sizes=ss)
        return y.numpy()

    res = a2a(comp.res_id.astype(np.int32), np.int32).astype(np.uint32)
    ts = a2a(comp.ts_ms, np.int64)
    cnt = a2a(comp.count, np.int32)
    fl = a2a(comp.flags.astype(np.int32), np.int32).astype(np.uint8)
    er = a2a(eref, np.int64)
    del comp, order, pos, eref
    part0 = np.concatenate([[0], np.cumsum(recv)])[:-1]
    part = np.repeat(np.arange(world), recv)
    er = np.where(er >= 0, er + part0[part], -1)             # index into the concatenation
    key = (ts - trace.T0).astype(np.uint16 if DURATION_MS < 65536 else np.uint32)
    mo = np.argsort(key, kind="stable")                      # time order; a millisecond keeps component order
    newpos = np.empty(mo.size, np.int64)
    newpos[mo] = np.arange(mo.size)
    er = er[mo]
    er = np.where(er >= 0, newpos[np.clip(er, 0, None)], -1)
    return abi.HostBatch(res[mo], ts[mo], cnt[mo], fl[mo], entry_ref=er), pl


def predict_ranks(args, steps=None, warmup=None):
    """The N-GPU run predicted on one GPU: the node-wide trace of bench.py's
    N-rank mode (N config-3 components of 2^27 events over all resources,
    seeds 3..3+N-1, merged in time order, hash-sharded res % N) is built on
    this host without a process group, and the shards of two ranks are timed
    like the headline step (HBM-resident, time-shifted batches pipelined): the
    rank holding the Zipf head (the most events) and the lightest one.  With
    weak scaling the N-rank step is the slowest rank's, so the implied 1 -> N
    efficiency is the single-GPU config-3 step over the head rank's step."""
    N, R = args.predict_ranks, args.resources
    steps, warmup = steps or args.steps, warmup or args.warmup
    t0 = time.time()
    grade_all, beh_all, count_all = trace.mixed_rule_table(R, seed=3)
    parts = {}
    counts = None
    node_entries = 0
    single = None
    for c in range(N):
        comp = trace.mixed_zipf(R, args.events, duration_ms=DURATION_MS, seed=3 + c)
        node_entries += int(((comp.flags & abi.EV_EXIT) == 0).sum())
        if c == 0:                                               # the single-GPU step of the same run
            single = time_shard(comp, abi.flow_rules_np(np.arange(R, dtype=np.uint32), grade_all, count_all,
                                                        beh_all), R, 1, 0, steps, warmup)
            log(f"[predict] single GPU: {single:.2f} ms/step")
        if c == 0:
            per0 = np.bincount(comp.res_id, minlength=R)
            sens = shard_share_sensitivity(per0, N)
            log(f"[predict] shard shares: {sens}")
            pl = None
            if args.placement:
                from sentinel_amd.placement import Placement
                pl = Placement.balanced(per0 * N, N, args.placement)   # (component 0 scaled: the previous batch)
            del per0
        eid = comp.res_id.astype(np.int64) if pl is None else pl.engine_id(comp.res_id)
        rk = eid % N
        if counts is None:
            counts = np.bincount(rk, minlength=N).astype(np.int64) * N       # (component 0 scaled: the choice)
            head = int(np.argmax(counts)); light = int(np.argmin(counts))
            # A resource is one serial chain on its rank whatever the placement: the
            # ranks that own the busiest THREAD / RateLimiter resource (k_heavy_stream)
            # and the busiest resource overall (k_heavy_decide) are timed as well.
            per0c = np.bincount(comp.res_id, minlength=R)
            stream_res = np.nonzero((grade_all == abi.GRADE_THREAD) | (beh_all == abi.BEHAVIOR_RATE_LIMITER))[0]
            chain = int(stream_res[np.argmax(per0c[stream_res])])
            top = int(np.argmax(per0c))
            del per0c
            own = (lambda r_: int(r_ % N)) if pl is None else (lambda r_: int(pl.owner(np.array([r_]))[0]))
            roles = {head: "head (most events)"}
            roles.setdefault(own(chain), f"owns the busiest THREAD / RateLimiter resource ({chain})")
            roles.setdefault(own(top), f"owns the busiest resource ({top})")
            roles.setdefault(light, "lightest")
            chosen = list(roles)
        for r in chosen:
            sel = np.nonzero(rk == r)[0]
            pos = np.full(comp.n, -1, np.int64)
            pos[sel] = np.arange(sel.size)
            er = comp.entry_ref[sel]
            er = np.where(er >= 0, pos[np.clip(er, 0, None)], -1)
            parts.setdefault(r, []).append((eid[sel].astype(np.uint32), comp.ts_ms[sel], comp.count[sel],
                                            comp.flags[sel], er))
        del comp, rk, eid
        log(f"[predict] component {c + 1}/{N} in {time.time() - t0:.0f}s")
    out = {"metric": METRIC, "mode": f"predict {N} ranks on one GPU", "n_ranks": N, "resources": R,
           "component_events": args.events, "steps": steps, "warmup": warmup, "ranks": {}}
    for r in chosen:
        ps = parts.pop(r)
        sizes = [p_[0].size for p_ in ps]
        off = np.concatenate([[0], np.cumsum(sizes)])[:-1]
        res = np.concatenate([p_[0] for p_ in ps]); ts = np.concatenate([p_[1] for p_ in ps])
        cnt = np.concatenate([p_[2] for p_ in ps]); fl = np.concatenate([p_[3] for p_ in ps])
        er = np.concatenate([np.where(p_[4] >= 0, p_[4] + o, -1) for p_, o in zip(ps, off)])
        del ps
        key = (ts - trace.T0).astype(np.uint16 if DURATION_MS < 65536 else np.uint32)
        mo = np.argsort(key, kind="stable")                      # time order; a millisecond keeps component order
        newpos = np.empty(mo.size, np.int64)
        newpos[mo] = np.arange(mo.size)
        er = er[mo]
        er = np.where(er >= 0, newpos[np.clip(er, 0, None)], -1)
        hb = abi.HostBatch(res[mo], ts[mo], cnt[mo], fl[mo], entry_ref=er)
        del res, ts, cnt, fl, er, mo, newpos, key
        if pl is None:
            mine = np.arange(r, R, N, dtype=np.int64)
            mine_eid, R_local = mine, (R - r + N - 1) // N
        else:
            mine = np.nonzero(pl.owner(np.arange(R)) == r)[0]
            mine_eid, R_local = pl.engine_id(mine), pl.local_rows()
        rules = abi.flow_rules_np(mine_eid.astype(np.uint32), grade_all[mine], count_all[mine], beh_all[mine])
        n_entry = int(((hb.flags & abi.EV_EXIT) == 0).sum())
        log(f"[predict] rank {r}: {hb.n} events, t={time.time() - t0:.0f}s")
        ms = time_shard(hb, rules, R_local, N, r, steps, warmup)
        out["ranks"][str(r)] = {"role": roles[r], "events": int(hb.n),
                                "entries": int(n_entry), "ms_per_step": round(ms, 3),
                                "events_vs_mean": round(hb.n / (N * args.events / N), 3)}
        log(f"[predict] rank {r}: {ms:.2f} ms/step")
        del hb
    out["expected_events_per_rank"] = {str(k): int(v) for k, v in enumerate(counts)}
    out["placement"] = None if pl is None else {
        "what": "top-K resources by component 0's counts spread LPT-greedy over the ranks, the rest at res % N "
                "(sentinel_amd/placement.py)", "K": int(pl.moved.size),
        "max_over_mean_events_expected": round(float(counts.max() / counts.mean()), 4)}
    head_ms = max(v["ms_per_step"] for v in out["ranks"].values())          # the slowest timed rank
    out["slowest_rank"] = max(out["ranks"], key=lambda k: out["ranks"][k]["ms_per_step"])
    out["single_gpu_ms_per_step"] = round(single, 3)
    out["node_step_ms"] = head_ms
    out["node_decisions_per_s"] = round(node_entries / (head_ms / 1e3), 1)
    out["implied_efficiency"] = round(single / head_ms, 4)
    # the same step under a hash of the resource name instead of the trace's
    # round-robin rank map: the head rank's time scaled by its share (time ~ events)
    out["shard_share"] = sens                    # (of the default map res % N)
    if pl is None:
        for q in ("p50", "p99"):
            f = sens[f"random_hash_max_share_{q}"] / sens["trace_map_max_share"]
            out[f"implied_efficiency_random_hash_{q}"] = round(single / (head_ms * f), 4)
    out["note"] = ("weak scaling: every rank decides its shard of one node-wide trace (N x 2^27 events); the node "
                   "step is the slowest rank's; implied efficiency = single-GPU step / slowest timed rank's step "
                   "(the ranks timed: most events, the owners of the busiest serial chains, the lightest)")
    print(json.dumps(out), flush=True)


def shard_share_sensitivity(per_res, N, K=1000, top=20000, seed=5):
    """How the busiest shard's share of the events depends on the id -> shard
    map.  trace.scramble maps popularity rank k to k * a mod R with a = 1 mod 8
    and 8 | R, so res % N == rank % N: the ranks are dealt round-robin, the
    head shard holds ranks 0, N, 2N, ...  A hash of the resource name (what
    a deployment shards by) deals the busiest resources at random instead.
    The max shard share for the trace's map and its distribution over K
    random assignments of the `top` busiest resources (the rest split evenly)."""
    per_res = np.asarray(per_res, np.float64)
    total = per_res.sum()
    order = np.argsort(-per_res)[:top]
    head = per_res[order]
    rest = (total - head.sum()) / N
    cur = np.bincount((order % N).astype(np.int64), weights=head, minlength=N) + rest
    rng = np.random.default_rng(seed)
    mx = np.empty(K)
    for k in range(K):
        mx[k] = (np.bincount(rng.integers(0, N, top), weights=head, minlength=N) + rest).max()
    return {"trace_map_max_share": round(float(cur.max() / total), 4),
            "random_hash_max_share_p50": round(float(np.percentile(mx, 50) / total), 4),
            "random_hash_max_share_p90": round(float(np.percentile(mx, 90) / total), 4),
            "random_hash_max_share_p99": round(float(np.percentile(mx, 99) / total), 4),
            "even_share": round(1.0 / N, 4)}


def time_shard(hb, rules, R_local, N, r, steps, warmup):
    """ms/step of one rank's shard: HBM-resident batches, pipelined as the headline run."""
    eng = engine.FlowEngine(abi.default_config(max_resources=R_local, max_batch=hb.n, shard_count=N, shard_index=r))
    try:
        eng.load_flow_rules(rules)
        base = engine.DeviceBatch(eng, hb)
        bl = [base] + [engine.DeviceBatch.with_ts(eng, base, hb.ts_ms + k * DURATION_MS)
                       for k in range(1, steps + warmup)]
        ov = engine.DeviceVerdicts(eng, hb.n, with_wait=True, with_rule=False)
        for k in range(warmup):
            eng.submit_device_async(bl[k], ov)
        eng.sync()
        t = time.perf_counter()
        for k in range(warmup, warmup + steps):
            eng.submit_device_async(bl[k], ov)
        eng.sync()
        ms = (time.perf_counter() - t) / steps * 1e3
        for b in bl:
            b.free()
        ov.free()
        return ms
    finally:
        eng.close()


def config3_origin_leg(hb, rules, R, c3_ms, steps=5, warmup=2, parity=True, n_origins=64,
                       variants=("no_origin_rules", "other_rules_1pct")):
    """Config 3 with a caller origin on every entry (ContextUtil.enter(name,
    origin)): one of 64 names drawn Zipf(1.1), exits carrying their entry's
    (trace.with_origins).  ClusterBuilderSlot creates the origin node of every
    entry with an origin (ClusterBuilderSlot.java:107-110), so every event also
    updates its (resource, origin) node.  Two variants, each on a fresh engine
    with HBM-resident batches pipelined like the headline run:
    ``no_origin_rules`` (the config-3 rules: the origin-node pass after the
    verdicts, sf_origin.hip) and ``other_rules_1pct`` (a limitApp "other" QPS
    rule added on 1 % of the resources, chosen by hash: those resources read
    origin nodes and run on the xflow walk).  ms/step is compared with the
    headline config-3 step of the same run.  Parity: every verdict of batch 0
    and of the last timed batch, and a sample of origin nodes (every origin of
    the 16 busiest resources, 512 random pairs), ClusterNodes and ENTRY_NODE
    after batch 0 and after the last batch, against the resource-sharded
    oracle replaying the same batches."""
    t0 = time.time()
    ho = trace.with_origins(hb, n_origins=n_origins, seed=13)
    log(f"[leg config3_origin] origins drawn in {time.time() - t0:.1f}s")
    res_local = ho.res_id
    per_res = np.bincount(res_local, minlength=R)
    key = res_local.astype(np.uint64) << np.uint64(32) | ho.origin.astype(np.uint64)
    busiest = np.argsort(-per_res)[:16]
    rng = np.random.default_rng(17)
    pick = rng.choice(ho.n, size=512, replace=False)
    bsel = np.isin(res_local, busiest)
    pairs = np.unique(np.concatenate([np.unique(key[bsel]), key[pick]]))
    pairs = [(int(k >> np.uint64(32)), int(k & np.uint64(0xffffffff))) for k in pairs]
    n_pairs = int(np.unique(key).size)
    del key
    node_sample = np.unique(np.concatenate([busiest, rng.choice(np.nonzero(per_res)[0], 256, replace=False)]))
    out = {"what": "config3 + a Zipf(1.1) origin out of 64 on every entry (origin nodes, ClusterBuilderSlot.java:107-110)",
           "events": int(ho.n), "distinct_pairs": n_pairs, "config3_ms_per_step": round(c3_ms, 3)}
    h = ((np.arange(R, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(40)) % np.uint64(100)
    xres = np.nonzero(h == 7)[0].astype(np.uint32)
    other = np.zeros(xres.size, abi.FLOW_RULE_DTYPE)
    other["resource"] = xres
    other["grade"] = abi.GRADE_QPS
    other["count"] = (20 + (xres % 200)).astype(np.float64)
    other["limit_app"] = abi.APP_OTHER
    other["warm_up_period_sec"] = 10
    other["max_queueing_time_ms"] = 500
    both = np.concatenate([rules, other])
    both = both[np.argsort(both["resource"], kind="stable")]    # per resource: the config-3 rule, then "other"
    for name, rl in (("no_origin_rules", rules), ("other_rules_1pct", both)):
        if name not in variants:
            continue
        e = engine.FlowEngine(abi.default_config(max_resources=R, max_batch=ho.n))
        res = {"rules": int(len(rl))}
        try:
            e.load_flow_rules(rl)
            base = engine.DeviceBatch(e, ho)
            n_b = warmup + steps
            bl = [base] + [engine.DeviceBatch.with_ts(e, base, ho.ts_ms + k * DURATION_MS) for k in range(1, n_b)]
            out0 = engine.DeviceVerdicts(e, ho.n, with_wait=True, with_rule=True)
            outv = engine.DeviceVerdicts(e, ho.n, with_wait=True, with_rule=True)
            t = time.perf_counter()
            e.submit_device_async(bl[0], out0)
            e.sync()
            res["batch0_ms"] = round((time.perf_counter() - t) * 1e3, 2)
            gpu0 = {"origin": [abi.node_state_to_dict(e.read_origin_node(r, o)) for r, o in pairs],
                    "nodes": [abi.node_state_to_dict(e.read_node(int(r))) for r in node_sample],
                    "entry": abi.node_state_to_dict(e.read_entry_node())}
            for k in range(1, warmup):
                e.submit_device_async(bl[k], outv)
            e.sync()
            e.set_timing(True)
            t = time.perf_counter()
            for k in range(warmup, n_b):
                e.submit_device_async(bl[k], outv)
            e.sync()
            ms = (time.perf_counter() - t) / steps * 1e3
            st = e.stats()
            res.update({"ms_per_step": round(ms, 3), "vs_config3": round(ms / c3_ms, 3),
                        "decisions_per_s": round(int(((ho.flags & abi.EV_EXIT) == 0).sum()) / (ms / 1e3), 1),
                        "origin_nodes": int(st.aux_nodes), "pool_capacity": int(st.aux_capacity),
                        "wave_walk": {"chunks_exact": int(st.xw_chunks_exact), "chunks_serial": int(st.xw_chunks_serial),
                                      "solve_rounds": int(st.xw_rounds), "serial_events": int(st.xw_serial_events)},
                        "index_grows": int(st.aux_index_grows)})
            log(f"[leg config3_origin] {name}: {ms:.2f} ms/step ({ms / c3_ms:.2f}x config 3), "
                f"{st.aux_nodes} origin nodes, wave walk {res['wave_walk']}")
            g0 = (out0.status.numpy(), out0.wait_ms.numpy(), out0.rule_idx.numpy())
            gl = (outv.status.numpy(), outv.wait_ms.numpy())
            gpu1 = {"origin": [abi.node_state_to_dict(e.read_origin_node(r, o)) for r, o in pairs],
                    "nodes": [abi.node_state_to_dict(e.read_node(int(r))) for r in node_sample],
                    "entry": abi.node_state_to_dict(e.read_entry_node())}
            for b in bl:
                b.free()
            out0.free(); outv.free()
        finally:
            e.close()
        if parity:
            try:
                from oracle import sharded
                from sentinel_amd import dist as sdist
                T = max(1, min(16, len(os.sched_getaffinity(0))))
                sh = sharded.ShardedOracle(rl, R, T, ho.n)
                sh.split_like(ho)
                log(f"[leg config3_origin] {name}: oracle replay of batch 0 ...")
                v, dt = sh.submit(ho)
                log(f"[leg config3_origin] {name}: oracle batch 0 in {dt:.1f}s")
                blk = np.isin(v.status, [abi.V_BLOCK_FLOW, abi.V_BLOCK_PARAM, abi.V_BLOCK_SYSTEM])
                mm = {"status": int((g0[0] != v.status).sum()), "wait_ms": int((g0[1] != v.wait_ms).sum()),
                      "rule_idx_of_blocks": int((g0[2][blk] != v.rule_idx[blk]).sum()),
                      "origin_nodes": sum(a != abi.node_state_to_dict(sh.read_origin_node(r, o))
                                          for a, (r, o) in zip(gpu0["origin"], pairs)),
                      "nodes": sum(a != abi.node_state_to_dict(sh.read_node(int(r)))
                                   for a, r in zip(gpu0["nodes"], node_sample)),
                      "entry_node": int(gpu0["entry"] != abi.node_state_to_dict(
                          sdist.merge_entry_nodes(sh.entry_nodes())))}
                res["cpu_baseline"] = {"value": round(int(((ho.flags & abi.EV_EXIT) == 0).sum()) / dt, 1),
                                       "unit": "decisions/s", "cores": T, "kind": "port",
                                       "sample": "batch 0, resource-sharded C oracle with origin nodes"}
                for k in range(1, warmup + steps):
                    v, dtk = sh.submit(ho, k * DURATION_MS)
                    log(f"[leg config3_origin] {name}: oracle batch {k} in {dtk:.1f}s")
                mm_last = {"status": int((gl[0] != v.status).sum()), "wait_ms": int((gl[1] != v.wait_ms).sum()),
                           "origin_nodes": sum(a != abi.node_state_to_dict(sh.read_origin_node(r, o))
                                               for a, (r, o) in zip(gpu1["origin"], pairs)),
                           "nodes": sum(a != abi.node_state_to_dict(sh.read_node(int(r)))
                                        for a, r in zip(gpu1["nodes"], node_sample)),
                           "entry_node": int(gpu1["entry"] != abi.node_state_to_dict(
                               sdist.merge_entry_nodes(sh.entry_nodes())))}
                sh.close()
                res["parity"] = {"what": f"batch 0 and batch {warmup + steps - 1} (every verdict; {len(pairs)} origin "
                                         f"nodes, {node_sample.size} ClusterNodes, ENTRY_NODE) vs the "
                                         f"resource-sharded oracle", "batch0": mm, "last": mm_last,
                                 "exact": all(x == 0 for x in mm.values()) and all(x == 0 for x in mm_last.values())}
            except Exception as ex:  # pragma: no cover
                res["parity"] = {"error": str(ex)[:200]}
        out[name] = res
    return out


def config2_leg(R=1_000_000, n=1 << 27, steps=3, parity=1):
    """BASELINE config 2 (its own engine): 1M resources, one QPS
    DefaultController rule each (count U{5..50}), a uniform trace of 2^27
    events per 4 s, HBM-resident batches decided back to back (async), and the
    roofline of the whole pipeline with SURVEY.md §8(d)'s byte model
    (25 B per event + 528 B per touched resource: 28.9 B per decision).
    Parity: batch 0 against the resource-sharded oracle."""
    counts = trace.uniform_rules(R)
    rules = abi.flow_rules_np(np.arange(R, dtype=np.uint32), np.full(R, abi.GRADE_QPS, np.int32), counts,
                              np.zeros(R, np.int32))
    hb = trace.uniform_qps(R, n)
    e = engine.FlowEngine(abi.default_config(max_resources=R, max_batch=hb.n))
    try:
        e.load_flow_rules(rules)
        base = engine.DeviceBatch(e, hb)
        bl = [base] + [engine.DeviceBatch.with_ts(e, base, hb.ts_ms + k * DURATION_MS) for k in range(1, steps + 1)]
        out0 = engine.DeviceVerdicts(e, hb.n, with_wait=True, with_rule=True)
        out = engine.DeviceVerdicts(e, hb.n, with_wait=True, with_rule=False)
        e.submit_device_async(bl[0], out0)
        e.sync()
        t = time.perf_counter()
        for k in range(1, steps + 1):
            e.submit_device_async(bl[k], out)
        e.sync()
        wall = (time.perf_counter() - t) / steps
        touched = int(np.count_nonzero(np.bincount(hb.res_id, minlength=R)))
        b_alg = 25 * hb.n + 528 * touched
        res = {"what": "config2: 1M resources uniform, QPS DefaultController (count U{5..50}), 2^27 events / 4 s, "
                       "HBM-resident, batches pipelined", "events_per_batch": int(hb.n), "resources_touched": touched,
               "ms_per_step": round(wall * 1e3, 3), "decisions_per_s": round(hb.n / wall, 1),
               "roofline": {"bound": "hbm", "what": "whole pipeline, SURVEY §8(d) byte model",
                            "alg_bytes_per_step": b_alg, "bytes_per_decision": round(b_alg / hb.n, 2),
                            "achieved": round(b_alg / wall / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(b_alg / wall / 1e9 / HBM_PEAK_GBS, 5)},
               "pass_fraction": round(float(np.isin(out.status.numpy(), abi.PASSED).mean()), 4)}
        try:
            if not parity:
                raise RuntimeError("parity leg skipped (parity=0)")
            from oracle import sharded
            g = out0.status.numpy()
            v, dt = sharded.replay(rules, hb, R, 16)
            res["parity"] = {"what": "batch 0 vs the resource-sharded oracle (16 threads)",
                             "mismatches": int((g != v.status).sum()), "exact": bool((g == v.status).all())}
            res["cpu_baseline"] = {"value": round(hb.n / dt, 1), "unit": "decisions/s", "cores": 16, "kind": "port",
                                   "sample": "batch 0, resource-sharded C oracle"}
        except Exception as ex:  # pragma: no cover
            res["parity"] = {"error": str(ex)[:200]}
        for b in bl:
            b.free()
        return res
    finally:
        e.close()


def system_exchange_leg(world, rank, device, dist, R=1000, n_per_rank=1 << 21, keys=1_000_000, qps_frac=0.6):
    """SystemRules on the sharded node (N > 1):
    config 4's shape over the whole node -- R x N resources with QPS /
    throttle ParamFlowRules, n x N events of Zipf(1.1) keys (weak scaling),
    the inbound-QPS SystemRule at qps_frac x the node's offered rate -- every
    rank deciding its shard res % N with sf_submit_node, the per-window
    exchange over RCCL (device buffers, ncclAllGather of 4224 B per rank and
    plan level).  Two runs on fresh engines, the second timed (barriers,
    max over ranks).  Rank 0 then decides the whole node batch on one engine
    (its GPU) and compares every verdict."""
    from sentinel_amd import dist as sdist
    RN, n = R * world, n_per_rank * world
    rules, b = trace.param_zipf(RN, n, keys, duration_ms=DURATION_MS, seed=4)
    sysr = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=qps_frac * n / (DURATION_MS / 1e3),
                               avg_rt=-1, max_thread=-1)]
    sel = np.nonzero(b.res_id % world == rank)[0]
    part = b.shard(world, rank)
    mine = [r for r in rules if r.resource % world == rank]
    cap = 1 << int(np.ceil(np.log2(max(8 * part.n, 1 << 16))))
    walls, v, st = [], None, None
    backend, comm = "rccl", None
    for rep in range(2):
        e = engine.FlowEngine(abi.default_config(max_resources=R, max_batch=part.n, shard_count=world,
                                                 shard_index=rank, device=device, param_capacity=cap))
        try:
            e.load_system_rules(sysr)
            e.load_param_rules(mine)
            if backend == "rccl":
                sys.stdout.flush()
                saved = os.dup(1)
                os.dup2(2, 1)              # RCCL's banner: stdout keeps the one JSON line
                try:
                    sdist.rccl_join(e)
                except engine.EngineError as ex:
                    # (ranks sharing one device -- the one-GPU rehearsal: RCCL refuses
                    # them; every rank alike, the communicator init is collective)
                    backend = f"gloo (RCCL refused: {str(ex)[:80]})"
                    from sentinel_amd import system_shard
                    comm = system_shard.TorchComm()
                finally:
                    os.dup2(saved, 1)
                    os.close(saved)
            dist.barrier()
            t = time.perf_counter()
            v = e.submit_node(part, sel, comm)
            wall = time.perf_counter() - t
            dist.barrier()
            walls.append(wall)
            st = e.stats()
        finally:
            e.close()
    import torch
    tt = torch.tensor([walls[-1]], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    ms = tt.item() * 1e3
    box = [None] * world if rank == 0 else None
    dist.gather_object((sel, v.status, v.wait_ms, v.rule_idx), box, dst=0)
    if rank != 0:
        return None
    got = np.full((3, b.n), -1, np.int64)
    for s_, a_, w_, r_ in box:
        got[:, s_] = np.stack([a_, w_, r_])
    e = engine.FlowEngine(abi.default_config(max_resources=RN, max_batch=b.n, device=device,
                                             param_capacity=1 << int(np.ceil(np.log2(max(8 * b.n, 1 << 16))))))
    try:
        e.load_system_rules(sysr)
        e.load_param_rules(rules)
        t = time.perf_counter()
        one = e.submit(b)
        one_ms = (time.perf_counter() - t) * 1e3
    finally:
        e.close()
    want = np.stack([one.status, one.wait_ms, one.rule_idx]).astype(np.int64)
    return {"what": f"config-4 shape on the sharded node: {RN} resources (ParamFlow, Zipf keys), {n} events, "
                    f"inbound QPS SystemRule at {qps_frac}x the node's offered rate; sf_submit_node per rank over "
                    "RCCL (per-window exchange, sf_sysx.h)", "ranks": world, "backend": backend,
            "ms_per_batch_max_over_ranks": round(ms, 3), "decisions_per_s": round(n / (ms / 1e3), 1),
            "planner_rounds": int(st.sys_rounds), "exchanges": int(st.sys_exchanges),
            "bytes_per_exchange_per_rank": 4224, "one_engine_whole_batch_ms": round(one_ms, 3),
            "system_blocks": int((want[0] == abi.V_BLOCK_SYSTEM).sum()),
            "parity": {"vs": "one engine deciding the whole node batch", "mismatches":
                       int((got != want).any(axis=0).sum()), "exact": bool((got == want).all())}}


def config4_leg(R=1000, n=1 << 24, keys=100_000_000, qps_frac=0.6, reps=3, parity=1):
    """BASELINE config 4 (its own engine): 1k resources with one QPS
    ParamFlowRule each (+10 % with a throttle rule), keys Zipf(1.1) over 100M
    distinct values, every event EntryType.IN, and the inbound-QPS SystemRule
    at qps_frac x the offered rate so that it blocks (the ParamFlow rules block
    ~21 %, so at 0.8x the SystemRule never fires).  One sf_submit of an
    HBM-resident batch from a fresh engine per rep; the planner cuts it into
    safe sub-batches (sf_system.h).  Parity: every verdict against the
    one-core oracle."""
    rules, b = trace.param_zipf(R, n, keys, duration_ms=DURATION_MS, seed=4)
    offered = b.n / (DURATION_MS / 1000.0)
    sysr = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=qps_frac * offered,
                               avg_rt=-1, max_thread=-1)]
    pairs = np.unique(b.res_id.astype(np.uint64) << np.uint64(40) ^ (b.arg_bits[0] & np.uint64((1 << 40) - 1))).size
    # the engine keeps room for every key a batch can insert (events x 2 x the
    # most rules on a resource, at half load: sf_engine.cpp param_reserve); a
    # table that large from the start keeps the rebuild out of the timed submit
    cap = 1 << int(np.ceil(np.log2(max(2 * b.n * 4, 2.5 * pairs * 1.1, 1 << 16))))
    cfg = abi.default_config(max_resources=R, max_batch=b.n, param_capacity=cap)
    walls, st, tab, rounds = [], None, None, 0
    log(f"[leg config4] trace {b.n} events, ~{pairs} (resource, key) pairs")
    for rep in range(reps):
        e = engine.FlowEngine(cfg)
        try:
            e.load_system_rules(sysr)
            e.load_param_rules(rules)
            db = engine.DeviceBatch(e, b)
            dv = engine.DeviceVerdicts(e, b.n, with_wait=True, with_rule=True)
            e.set_timing(True)
            e.sync()
            t = time.perf_counter()
            e.submit_device(db, dv)
            walls.append(time.perf_counter() - t)
            if rep == reps - 1:
                st = (dv.status.numpy(), dv.wait_ms.numpy(), dv.rule_idx.numpy())
                tab = e.param_table_stats()
                rounds = int(e.stats().sys_rounds)
            db.free()
            dv.free()
        finally:
            e.close()
    ms = 1e3 * float(np.median(walls))
    ent = int(((b.flags & abi.EV_EXIT) == 0).sum())
    res = {"what": f"config4: ParamFlow 100M-key Zipf(1.1) on {R} resources + SystemRule qps {qps_frac}x offered, "
                   f"one HBM-resident batch from a fresh engine", "events": int(b.n),
           "ms_per_batch": round(ms, 3), "decisions_per_s": round(ent / (ms / 1e3), 1),
           "planner_rounds": rounds, "distinct_pairs": int(pairs), "param_table": tab,
           "load_factor": round(tab["used"] / tab["capacity"], 4) if tab else None,
           "system_blocks": int((st[0] == abi.V_BLOCK_SYSTEM).sum()),
           "param_blocks": int((st[0] == abi.V_BLOCK_PARAM).sum()),
           "passed": int(np.isin(st[0], abi.PASSED).sum()), "reps_ms": [round(1e3 * w, 3) for w in walls]}
    if not parity:
        return res
    log(f"[leg config4] GPU {ms:.1f} ms per batch; oracle replays (exact maps, and LRU maps as the reference) ...")
    try:
        import threading
        from oracle import oracle as so

        def replay(lru, slot):
            o = so.OracleEngine(cfg)
            if lru:
                o.set_param_lru(True)           # ConcurrentLinkedHashMap capacities (ParameterMetric.java:37-39,99)
            o.load_system_rules(sysr)
            o.load_param_rules(rules)
            t = time.perf_counter()
            slot["v"] = o.submit(b)
            slot["dt"] = time.perf_counter() - t
            slot["lru"] = o.param_lru_stats() if lru else None
            o.close()

        ex, lr = {}, {}
        th = [threading.Thread(target=replay, args=(False, ex)), threading.Thread(target=replay, args=(True, lr))]
        for x in th:
            x.start()
        for x in th:
            x.join()
        want, ref = ex["v"], lr["v"]
        bad = {"status": int((st[0] != want.status).sum()), "wait_ms": int((st[1] != want.wait_ms).sum()),
               "rule_idx": int((st[2] != want.rule_idx).sum())}
        bad_ref = {"status": int((st[0] != ref.status).sum()), "wait_ms": int((st[1] != ref.wait_ms).sum()),
                   "rule_idx": int((st[2] != ref.rule_idx).sum())}
        res["parity"] = {"what": "every verdict vs the one-core oracle replay (exact maps, as the engine)",
                         "mismatches": bad, "exact": all(v == 0 for v in bad.values()),
                         "lru_divergent_verdicts": int((want.status != ref.status).sum()
                                                       + ((want.status == ref.status) & ((want.wait_ms != ref.wait_ms)
                                                                                         | (want.rule_idx != ref.rule_idx))).sum()),
                         "lru_evictions": lr["lru"][0], "lru_spins": lr["lru"][1],
                         "vs_lru_reference": {"what": "every verdict vs the oracle with ParameterMetric's maps as the "
                                                     "reference's LRUs (capacity min(4000*durationInSec, 200000) = 4000)",
                                              "mismatches": bad_ref, "exact": all(v == 0 for v in bad_ref.values())}}
        res["cpu_baseline"] = {"value": round(ent / ex["dt"], 1), "unit": "decisions/s", "cores": 1, "kind": "port",
                               "sample": "the whole batch, one-core C oracle (exact maps)"}
    except Exception as ex:  # pragma: no cover
        res["parity"] = {"error": str(ex)[:200]}
    return res


def config5_leg(n_req=1 << 22, n_streams=500, steps=3):
    """BASELINE config 5 (its own engine): the cluster token server for 500
    client connections -- 10k flow rules + 1k param rules (Zipf(1.1) values
    over 1M), 10 % prioritized, namespace limiter open.  sf_serve_frames: the
    raw C1 request frames of all connections in, response frames out (device
    clock, framing to encoded responses); sf_request_tokens: the same requests
    as a token batch (wall clock incl. PCIe).  Parity: a 64k-request instance
    replayed through the oracle's wire path, every response byte compared."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import wire_bench
    ns, flow, param, streams = wire_bench.frames(n_req, n_streams, 7)
    cfg = abi.default_config(max_resources=4, max_batch=n_req, param_capacity=1 << 22)
    cfg.max_flow_ids = 1 << 15
    e = engine.FlowEngine(cfg)
    try:
        e.load_namespaces(ns)
        e.load_cluster_rules(flow, param, [])
        e.serve_frames(streams, trace.T0)
        e.set_timing(True)
        dev, wall = [], []
        for k in range(steps):
            t = time.perf_counter()
            r = e.serve_frames(streams, trace.T0 + 1000 * (k + 1))
            wall.append(time.perf_counter() - t)
            dev.append(e.stats().wire_ms)
        n_bytes = sum(len(x) for x in streams)
        ms = float(np.median(dev))
        res = {"what": "config5: cluster token server, 500 connections, C1 frames -> DefaultTokenService -> frames",
               "requests": int(r.n_requests), "in_bytes": int(n_bytes), "out_bytes": int(r.n_responses) * 16,
               "serve_frames": {"device_ms": round(ms, 3), "requests_per_s": round(r.n_requests / (ms / 1e3), 1),
                                "wall_ms_incl_pcie": round(float(np.median(wall)) * 1e3, 2)}}
    finally:
        e.close()
    # sf_request_tokens on a decoded batch of the same shape
    tns, tflow, tparam, titems, tbatch = trace.token_workload(n_req, n_flow=10_000, n_param=1000, n_values=1 << 20,
                                                              connected=n_streams, max_qps=1e12)
    cfg3 = abi.default_config(max_resources=4, max_batch=n_req, param_capacity=1 << 22)
    cfg3.max_flow_ids = 1 << 15
    e = engine.FlowEngine(cfg3)
    try:
        e.load_namespaces(tns)
        e.load_cluster_rules(tflow, tparam, titems)
        w = []
        for k in range(steps):
            tb = abi.HostTokenBatch(tbatch.flow_id, tbatch.count, tbatch.flags, tbatch.ts_ms + k * DURATION_MS,
                                    param_tag=tbatch.param_tag, param_bits=tbatch.param_bits)
            t = time.perf_counter()
            e.request_tokens(tb)
            w.append(time.perf_counter() - t)
        ms = float(np.median(w)) * 1e3
        res["request_tokens"] = {"requests": int(tbatch.n), "wall_ms_incl_pcie": round(ms, 3),
                                 "requests_per_s": round(tbatch.n / (ms / 1e3), 1)}
    except Exception as ex:  # pragma: no cover
        res["request_tokens"] = {"error": str(ex)[:200]}
    finally:
        e.close()
    try:
        # parity on the benchmarked frames themselves: all requests, a fresh
        # engine and a fresh oracle wire path, every response frame compared
        from oracle import oracle as so
        cfg2 = abi.default_config(max_resources=4, max_batch=n_req, param_capacity=1 << 22)
        cfg2.max_flow_ids = 1 << 15
        g = engine.FlowEngine(cfg2)
        o = so.OracleEngine(cfg2)
        for x in (g, o):
            x.load_namespaces(ns)
            x.load_cluster_rules(flow, param, [])
        t = time.perf_counter()
        rg = g.serve_frames(streams, trace.T0)
        ro = o.serve_frames(streams, trace.T0)
        t_or = time.perf_counter() - t
        bad = sum(rg.responses(s) != ro.responses(s) for s in range(n_streams))
        g.close()
        o.close()
        res["parity"] = {"what": f"all {int(ro.n_requests)} requests of the benchmarked frames over {n_streams} "
                                 f"connections, fresh engine and fresh oracle wire path: every response frame",
                         "requests": int(ro.n_requests), "connections_differing": int(bad), "exact": bad == 0,
                         "seconds": round(t_or, 1)}
    except Exception as ex:  # pragma: no cover
        res["parity"] = {"error": str(ex)[:200]}
    return res


def e2e_leg(hb, rules, R, steps, g0, glast, timed=None):
    """Both compact forms: the narrow 4-byte words (resource ids below 2^24,
    the time as a per-millisecond table; the line's numbers) and the 8-byte
    words the Java shim sends (its numbers under form_8byte)."""
    narrow = int(hb.res_id.max()) < (1 << 24)
    out = e2e_form(hb, rules, R, steps, g0, glast, timed, narrow=narrow)
    if narrow:
        w = e2e_form(hb, rules, R, steps, g0, glast, timed, narrow=False)
        out["form_8byte"] = {k: w[k] for k in ("ms_per_batch", "decisions_per_s", "latency_ms", "period_ms",
                                               "h2d_bytes", "h2d_alone_ms", "period_over_h2d", "parity")}
    return out


def e2e_form(hb, rules, R, steps, g0, glast, timed=None, narrow=False):
    """Config 3 end to end from page-locked host memory: the headline run's
    batches (the same trace, shifted by DURATION_MS per step) submitted from
    host buffers in the compact form (sf_submit_packed_async: 8 bytes per event
    plus the exits' entry refs), so that the H2D copy of batch k+1, the
    decision of batch k and the D2H copy of the verdicts (status, wait, rule
    index) of batch k-1 overlap.  A fresh engine; the time shift is only the
    batch's ts_base, so every step reuses the same pinned words.  Parity: the
    verdicts of batch 0 and of the last batch equal the headline run's (itself
    compared with the oracle).  PCIe-inclusive: never the headline."""
    e = engine.FlowEngine(abi.default_config(max_resources=R, max_batch=hb.n))
    pin = engine.PinnedArrays(e)
    try:
        e.load_flow_rules(rules)
        t0 = time.perf_counter()
        pb = abi.PackedBatch(hb, alloc=pin.array, narrow=narrow)
        log(f"[leg e2e_pinned] {'narrow ' if narrow else ''}packed {hb.n} events into {pb.nbytes() / 1e9:.2f} GB in {time.perf_counter() - t0:.1f}s")
        # sparse copy back (sf_submit_packed_sparse_async): 1 status byte per event plus
        # the nonzero waits / rule indices, n/64 entries of each list prefetched with it
        # (config 3 queues 1.3 % of its events; a longer list is completed at the sync)
        pre = hb.n // 64
        outs = [pin.sparse_verdicts(hb.n, pre) for _ in range(3)]
        base_ts = pb.ts_base
        timed = timed or max(3, steps - 2)
        walls = []
        t = None
        for k in range(steps):
            if k == steps - timed:
                e.sync()
                t = time.perf_counter()
            pb.ts_base = base_ts + k * DURATION_MS
            o = outs[0] if k == 0 else (outs[1] if k == steps - 1 else outs[2])
            e.submit_packed_sparse_async(pb, o)
            if k == 0:
                e.sync()                                   # batch 0 kept for parity
        e.sync()
        total = time.perf_counter() - t
        ms = total / timed * 1e3
        # one batch alone (its latency: H2D, decision, D2H in sequence); the
        # steady-state period of the pipeline is the rest over timed - 1 batches
        pb.ts_base = base_ts + steps * DURATION_MS
        t1 = time.perf_counter()
        e.submit_packed_sparse_async(pb, outs[2])
        e.sync()
        lat = time.perf_counter() - t1
        period = (total - lat) / max(1, timed - 1) * 1e3
        ent = int(((hb.flags & abi.EV_EXIT) == 0).sum())
        # the H2D-bound time: the packed arrays copied alone (pinned -> HBM, synchronous)
        import ctypes as C
        arrs = [a for a in (pb.ev, pb.ev4, pb.ms_end, pb.exit_ref, pb.exit_cts, pb.count_ext, pb.origin)
                if a is not None and a.nbytes]
        dptr = C.c_void_p()
        engine._check(engine.lib().sf_device_alloc(e.h, max(a.nbytes for a in arrs), C.byref(dptr)))
        h2d = []
        for _ in range(3):
            t2 = time.perf_counter()
            for a in arrs:
                engine._check(engine.lib().sf_memcpy(e.h, dptr.value, a.ctypes.data, a.nbytes, 0))
            h2d.append(time.perf_counter() - t2)
        engine._check(engine.lib().sf_device_free(e.h, dptr.value))
        h2d_ms = 1e3 * min(h2d)
        d0, dl = outs[0].dense(), outs[1].dense()
        bad0 = {"status": int((d0.status != g0[0]).sum()), "wait_ms": int((d0.wait_ms != g0[1]).sum()),
                "rule_idx": int((d0.rule_idx != g0[2]).sum())}
        badl = {"status": int((dl.status != glast[0]).sum()), "wait_ms": int((dl.wait_ms != glast[1]).sum())}
        lists = [int(outs[1].counts[0]), int(outs[1].counts[1])]
        d2h = int(hb.n + 8 + 2 * 8 * pre + 8 * sum(max(0, c - pre) for c in lists))
        return {"what": "config3 batches from pinned host buffers in the compact form (sf_submit_packed_sparse_async: "
                        "H2D of batch k+1, decide of k and the sparse D2H of k-1 overlapped)",
                "form": "narrow: 4 B per event + per-ms time table" if narrow else "8 B per event",
                "events": int(hb.n), "ms_per_batch": round(ms, 3), "decisions_per_s": round(ent / (ms / 1e3), 1),
                "latency_ms": round(lat * 1e3, 3), "period_ms": round(period, 3),
                "period_note": "ms_per_batch includes the drain of the last batch; period_ms = (timed wall - one "
                               "batch's latency) / (timed - 1), the steady-state interval of the pipeline",
                "timed_batches": timed, "h2d_bytes": int(pb.nbytes()), "d2h_bytes": d2h,
                "d2h_bytes_per_event": round(d2h / hb.n, 3), "d2h_dense_bytes": int(hb.n * (1 + 4 + 2)),
                "h2d_alone_ms": round(h2d_ms, 3), "period_over_h2d": round(period / h2d_ms, 3),
                "sparse_lists": {"waits": lists[0], "rules": lists[1], "prefetch_each": pre},
                "parity": {"what": "batch 0 and the last batch vs the headline run's verdicts", "batch0": bad0,
                           "last": badl, "exact": all(v == 0 for v in bad0.values()) and
                           all(v == 0 for v in badl.values())}}
    finally:
        pin.free()
        e.close()


def degrade_leg(R=1_000_000, entries=1 << 22, steps=3):
    """sf_degrade_submit over an HBM-resident batch: one circuit breaker (RT /
    exception ratio / exception count) on half of 1M resources, Zipf(1.1)
    entries each followed by its exit; every step replays from fresh breakers."""
    rules = trace.degrade_rules_array(R, seed=5)
    b = trace.degrade_workload(R, entries, duration_ms=4000, seed=6, s=1.1)
    e = engine.FlowEngine(abi.default_config(max_resources=R, max_batch=b.n))
    try:
        n_cb = e.load_degrade_rules(rules)
        db = engine.DeviceBatch(e, b)
        # every step replays the trace from fresh breakers (an empty load drops
        # them; an equal rule would keep its breaker), shifted by a multiple of
        # every stat interval so the clock moves forward and verdicts repeat
        span = (int(b.ts_ms[-1] - b.ts_ms[0]) // 60_000 + 2) * 60_000
        dbs = [engine.DeviceBatch.with_ts(e, db, b.ts_ms + k * span) for k in range(1, steps + 1)]
        dv = engine.DeviceVerdicts(e, b.n, with_wait=False, with_rule=True)
        e.degrade_submit_device(db, dv)
        wall = []
        for k in range(steps):
            e.load_degrade_rules([])
            e.load_degrade_rules(rules)
            t = time.perf_counter()
            e.degrade_submit_device(dbs[k], dv)
            wall.append(time.perf_counter() - t)
        for x in dbs:
            x.free()
        ms = float(np.median(wall)) * 1e3
        st = dv.status.numpy()
        db.free()
        return {"what": "DegradeSlot circuit breakers (sf_degrade_submit), Zipf(1.1), fresh breakers per step",
                "resources": R, "breakers": int(n_cb), "events": int(b.n), "ms_per_batch": round(ms, 3),
                "events_per_s": round(b.n / (ms / 1e3), 1),
                "blocked": int((st == abi.V_BLOCK_DEGRADE).sum())}
    finally:
        e.close()


def metric_log_leg(eng, hb, R_total, R_local, world, rank, steps, res_of_eid=None):
    """Resource names "/r/NNNNNNNN" (global id) and types, indexed by engine id
    (res_of_eid: a placement's inverse map); a drain fetch at
    T_last + 2 s (cap 0: rows counted, lastFetchTime advanced, nothing
    copied), then the timed fetch at T_last + 3 s: the second [T_last + 2 s,
    T_last + 3 s) of every node (and ENTRY_NODE), formatted as metrics.log."""
    ids = np.arange(R_total, dtype=np.int64) if res_of_eid is None else np.maximum(res_of_eid, 0)
    n_ids = ids.size
    digits = ((ids[:, None] // (10 ** np.arange(7, -1, -1))) % 10 + 48).astype(np.uint8)
    names = np.concatenate([np.frombuffer(b"/r/" * n_ids, np.uint8).reshape(n_ids, 3), digits], axis=1)
    off = np.arange(n_ids + 1, dtype=np.uint64) * 11
    eng.load_resource_names_raw(names.tobytes(), off, (ids % 3).astype(np.int32))
    t_last = int(hb.ts_ms[0]) + (steps - 1) * DURATION_MS
    try:
        eng.metric_log(t_last + 2000, entry_node=(rank == 0), cap=0)
    except engine.EngineError as ex:
        if ex.code != abi.SF_ERR_CAPACITY:
            raise
    import ctypes
    buf = ctypes.create_string_buffer(1 << 30)
    t = time.perf_counter()
    data = eng.metric_log(t_last + 3000, entry_node=(rank == 0), cap=1 << 30, buf=buf)
    wall_ms = (time.perf_counter() - t) * 1e3
    st = eng.stats()
    nodes = R_local + (1 if rank == 0 else 0)
    scan_bytes = 3840 * nodes                       # the 60 x 64 B minute row metrics() walks per node
    ach = scan_bytes / (st.metric_scan_ms / 1e3) / 1e9
    return {"what": "MetricTimerListener.run -> metrics.log lines (one second)", "nodes": nodes,
            "lines": data.count(b"\n"), "log_bytes": len(data), "device_ms": round(st.metric_log_ms, 3),
            "wall_ms_incl_d2h": round(wall_ms, 3),
            "scan": {"kernel": "k_mlog_count", "ms": round(st.metric_scan_ms, 3), "alg_bytes": scan_bytes,
                     "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4)},
            "sample_line": data[:data.find(b"\n")].decode(errors="replace") if data else ""}


def oracle_leg(rules, hb, R, out0, out_last, eng, steps, per_res):
    """The C restatement (oracle/, test infrastructure only).

    1. One core replays batch 0 from fresh state: verdicts compared with the
       GPU's batch 0 (status, wait, rule index of blocks); its time is the
       one-core CPU baseline.
    2. The resource-sharded oracle (one OracleEngine per res % T shard on T
       host threads, oracle/sharded.py) replays every batch of the run in
       order -- the same trace shifted by DURATION_MS per step, state carried
       across batches (minute buckets reused after the 60 s wrap, RateLimiter
       latestPassedTime, WarmUp tokens).  Batch 0's replay time is the
       multi-core CPU baseline (its verdicts must equal the one-core replay);
       the last batch's verdicts (status, wait) are compared with the GPU's
       last timed batch, and so are the node state (per-row digests) and the
       controller state of every resource and ENTRY_NODE."""
    try:
        from oracle import oracle as so
        from oracle import sharded
    except Exception as ex:  # pragma: no cover
        return {"error": str(ex)}, {"error": str(ex)}
    ora = so.OracleEngine(abi.default_config(max_resources=R, max_batch=hb.n))
    t = time.perf_counter()
    ora.load_flow_rules(rules)
    t_load = time.perf_counter() - t
    log("[oracle] one-core replay of batch 0 ...")
    t = time.perf_counter()
    want = ora.submit(hb)
    dt = time.perf_counter() - t
    log(f"[oracle] one-core replay of batch 0: {dt:.1f}s")
    ent = int(((hb.flags & abi.EV_EXIT) == 0).sum())
    ora.close()
    st, wt, ru = out0.status.numpy(), out0.wait_ms.numpy(), out0.rule_idx.numpy()
    blk = np.isin(want.status, [abi.V_BLOCK_FLOW, abi.V_BLOCK_PARAM, abi.V_BLOCK_SYSTEM])
    mism = {"status": int((st != want.status).sum()), "wait_ms": int((wt != want.wait_ms).sum()),
            "rule_idx_of_blocks": int((ru[blk] != want.rule_idx[blk]).sum())}
    single = {"value": round(ent / dt, 1), "unit": "decisions/s", "cores": 1, "kind": "port",
              "sample": f"the whole batch 0 ({hb.n} events, {ent} entries) of the timed workload from fresh state, "
                        f"single-threaded C oracle (rule load {t_load:.1f}s excluded)", "seconds": round(dt, 2)}
    cpu = single
    steady = None
    try:
        try:
            ncore = len(os.sched_getaffinity(0))
        except AttributeError:  # pragma: no cover
            ncore = os.cpu_count() or 1
        T = max(1, min(16, ncore))                       # the box's CPU share is 16
        sh = sharded.ShardedOracle(rules, R, T, hb.n)
        sh.split_like(hb)
        t_all = time.perf_counter()
        for k in range(steps):
            v, dtk = sh.submit(hb, k * DURATION_MS)
            log(f"[oracle] sharded replay of batch {k}: {dtk:.1f}s")
            if k == 0:
                same = bool((v.status == want.status).all() and (v.wait_ms == want.wait_ms).all())
                cpu = {"value": round(ent / dtk, 1), "unit": "decisions/s", "cores": T, "kind": "port",
                       "sample": f"the whole batch 0 ({hb.n} events, {ent} entries) split by resource (res % {T}) "
                                 f"over {T} threads, one C oracle per shard, verdicts merged (equal to the one-core "
                                 f"replay: {same})", "seconds": round(dtk, 2), "single_core": single}
        t_all = time.perf_counter() - t_all
        gs, gw = out_last.status.numpy(), out_last.wait_ms.numpy()
        # every node and every rule's controller state: the engine's per-row
        # digests (sf_node_digests, on the device) against the oracle shards'
        t_d = time.perf_counter()
        node_bad = int((eng.node_digests(R) != sh.node_digests(R)).sum())
        rule_bad = int((eng.rule_states(0, R) != sh.rule_states(R)).any(axis=1).sum())
        log(f"[oracle] whole-node comparison: {node_bad} node / {rule_bad} rule-state mismatches "
            f"in {time.perf_counter() - t_d:.1f}s")
        from sentinel_amd import dist as sdist
        en_same = abi.node_state_to_dict(eng.read_entry_node()) == \
            abi.node_state_to_dict(sdist.merge_entry_nodes(sh.entry_nodes()))
        sh.close()
        lm = {"status": int((gs != v.status).sum()), "wait_ms": int((gw != v.wait_ms).sum()),
              "nodes": node_bad, "rule_states": rule_bad, "entry_node": 0 if en_same else 1}
        steady = {"what": f"every batch of the run ({steps}: warmup + timed, state carried across batches, "
                          f"{steps * DURATION_MS // 1000} s of trace time) replayed by the resource-sharded oracle; "
                          f"batch {steps - 1} (the last timed one) compared",
                  "batch": steps - 1, "events": int(hb.n), "nodes_compared": int(R), "rule_states_compared": int(R),
                  "how": "every resource's node (FNV-1a 64 digest of its canonical sf_node_state, sf_node_digests "
                         "vs so_node_digests) and every rule's controller state, plus ENTRY_NODE",
                  "mismatches": lm, "exact": all(x == 0 for x in lm.values()), "replay_s": round(t_all, 1)}
    except Exception as ex:  # pragma: no cover - the one-core figure stays
        cpu = dict(single, multicore_error=str(ex)[:200])
        steady = {"error": str(ex)[:200]}
    parity = {"what": "batch 0 of the timed run (fresh engine) vs the oracle replay of the same batch",
              "events": int(hb.n), "mismatches": mism,
              "exact": all(v == 0 for v in mism.values()), "steady_state": steady}
    return cpu, parity


if __name__ == "__main__":
    main()
