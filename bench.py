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
    ap.add_argument("--heavy-min", type=int, default=0,
                    help="segments of more events than this go to the heavy kernels (0: the engine default, 512)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    assert world == args.gpus or world == 1, "launch N>1 with torch.distributed.run"

    R_total = args.resources
    R_local = (R_total - rank + world - 1) // world
    t0 = time.time()
    grade, beh, count = trace.mixed_rule_table(R_local, seed=3 + rank)
    rules = abi.flow_rules_np(np.arange(R_local, dtype=np.uint32) * world + rank, grade, count, beh)
    hb = trace.mixed_zipf(R_local, args.events, duration_ms=DURATION_MS, seed=3 + rank)
    hb.res_id = (hb.res_id.astype(np.uint64) * world + rank).astype(np.uint32)
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
    profs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_config3_summary.json")))
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
    roofline = {"bound": "hbm", "kernel": name, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "traffic_source": traffic_src,
                "alg_bytes_per_launch": bytes_k, "avg_launch_ms": round(ms, 4),
                "light_phase": light_phase,
                "pipeline": {"alg_bytes_per_step": b_alg,
                             "achieved_GBs": round(b_alg / (wall / k) / 1e9, 2),
                             "heavy_segments": n_heavy_res},
                "kernels_ms": {"sort+segments+classify": round(st.sort_ms / k, 3),
                               "classify": round(st.classify_ms / k, 3),
                               "decide(join)": round(st.decide_ms / k, 3),
                               "k_decide_light": round(st.light_ms / k, 3),
                               "k_heavy_decide": round(st.heavy_decide_ms / k, 3),
                               "k_heavy_stream": round(st.stream_ms / k, 3),
                               "k_heavy_fill": round(st.heavy_fill_ms / k, 3),
                               "scatter": round(st.scatter_ms / k, 3)}}

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
            metric_log = metric_log_leg(eng, hb, R_total, R_local, world, rank, steps)
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

    # whole-batch parity (batch 0 from a fresh engine vs the oracle replaying
    # the same batch) -- the same replay, timed, is the CPU baseline
    cpu, parity = None, None
    if rank == 0 and world == 1 and not args.no_cpu and args.warmup > 0:
        cpu, parity = oracle_leg(rules, hb, R_local, out0)

    if rank == 0:
        line = {"metric": METRIC, "value": round(value, 1), "unit": "decisions/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
                "data": "synthetic",
                "config": {"workload": "config3: 10M resources Zipf(1.1), 60% QPS / 10% THREAD / 15% WarmUp / "
                                       "15% RateLimiter, acquireCount 1 (90%) or 2-5, RT~Exp(20ms) exits",
                           "resources": R_total, "events_per_batch_per_gpu": hb.n, "entries_per_batch_per_gpu": n_entry,
                           "resources_touched": n_seg, "pass_fraction": round(n_pass / max(1, n_entry), 4),
                           "parallelism": f"resource-sharded x{world}"},
                "roofline": roofline, "cpu_baseline": cpu, "parity": parity, "aggregate": aggregate,
                "metric_log": metric_log, "degrade": degrade}
        print(json.dumps(line), flush=True)
    for b in batches[1:]:
        b.free()
    base.free()
    if dist:
        dist.destroy_process_group()


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


def metric_log_leg(eng, hb, R_total, R_local, world, rank, steps):
    """Resource names "/r/NNNNNNNN" (global id) and types; a drain fetch at
    T_last + 2 s (cap 0: rows counted, lastFetchTime advanced, nothing
    copied), then the timed fetch at T_last + 3 s: the second [T_last + 2 s,
    T_last + 3 s) of every node (and ENTRY_NODE), formatted as metrics.log."""
    ids = np.arange(R_total, dtype=np.int64)
    digits = ((ids[:, None] // (10 ** np.arange(7, -1, -1))) % 10 + 48).astype(np.uint8)
    names = np.concatenate([np.frombuffer(b"/r/" * R_total, np.uint8).reshape(R_total, 3), digits], axis=1)
    off = np.arange(R_total + 1, dtype=np.uint64) * 11
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


def oracle_leg(rules, hb, R, out0):
    """The C restatement (oracle/, test infrastructure) replays the whole
    batch 0 on one host core from fresh state: its verdicts are compared with
    the GPU's verdicts of that batch (status, wait, rule index: parity), and
    its time is the CPU baseline."""
    try:
        from oracle import oracle as so
    except Exception as ex:  # pragma: no cover
        return {"error": str(ex)}, {"error": str(ex)}
    ora = so.OracleEngine(abi.default_config(max_resources=R, max_batch=hb.n))
    t = time.perf_counter()
    ora.load_flow_rules(rules)
    t_load = time.perf_counter() - t
    t = time.perf_counter()
    want = ora.submit(hb)
    dt = time.perf_counter() - t
    ent = int(((hb.flags & abi.EV_EXIT) == 0).sum())
    ora.close()
    st, wt, ru = out0.status.numpy(), out0.wait_ms.numpy(), out0.rule_idx.numpy()
    blk = np.isin(want.status, [abi.V_BLOCK_FLOW, abi.V_BLOCK_PARAM, abi.V_BLOCK_SYSTEM])
    mism = {"status": int((st != want.status).sum()), "wait_ms": int((wt != want.wait_ms).sum()),
            "rule_idx_of_blocks": int((ru[blk] != want.rule_idx[blk]).sum())}
    single = {"value": round(ent / dt, 1), "unit": "decisions/s", "cores": 1, "kind": "port",
              "sample": f"the whole batch 0 ({hb.n} events, {ent} entries) of the timed workload from fresh state, "
                        f"single-threaded C oracle (rule load {t_load:.1f}s excluded)", "seconds": round(dt, 2)}
    # the multi-core CPU baseline: the same batch split by resource
    # over the box's cores, one oracle per shard (oracle/sharded.py)
    cpu = single
    try:
        from oracle import sharded
        try:
            ncore = len(os.sched_getaffinity(0))
        except AttributeError:  # pragma: no cover
            ncore = os.cpu_count() or 1
        T = max(1, min(16, ncore))                       # the box's CPU share is 16
        got, dtm = sharded.replay(rules, hb, R, T)
        same = bool((got.status == want.status).all() and (got.wait_ms == want.wait_ms).all())
        cpu = {"value": round(ent / dtm, 1), "unit": "decisions/s", "cores": T, "kind": "port",
               "sample": f"the whole batch 0 ({hb.n} events, {ent} entries) split by resource (res % {T}) over {T} "
                         f"threads, one C oracle per shard, verdicts merged (equal to the one-core replay: {same})",
               "seconds": round(dtm, 2), "single_core": single}
    except Exception as ex:  # pragma: no cover - the one-core figure stays
        cpu = dict(single, multicore_error=str(ex)[:200])
    parity = {"what": "batch 0 of the timed run (fresh engine) vs the oracle replay of the same batch",
              "events": int(hb.n), "mismatches": mism,
              "exact": all(v == 0 for v in mism.values())}
    return cpu, parity


if __name__ == "__main__":
    main()
