#!/usr/bin/env python3
"""Headline benchmark: env-steps/s of the vectorised LB environment (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--servers S]

One rank per GPU: under torch.distributed.run, or, for --gpus N > 1 without it, N rank processes
this script starts itself (same environment contract).  Weak scaling: every GPU steps its own shard of B envs
(global ids [rank*B, (rank+1)*B) key the RNG, so shards never communicate); the only collectives
are the timing barrier and the max/sum reductions of the result.  A "step" is one VecEnv.step of
every env: random-policy actions drawn on the GPU, dynamics kernel, observe kernel (features,
reward, done), episode bookkeeping and the masked auto-reset launch.

Default N=1 workload: 65536 envs x 4 servers (north-star point; BASELINE configs[1] is the same
random-policy rollout at 4096 envs and is a parity-test case).  Prints ONE JSON line (rank 0)
with a `roofline` object for the dominant kernel (HIP-event timed inside the timed region), a
`cpu_baseline` (the C oracle on host cores, bounded sample of the same workload) and, with
`--late-episode 1000,5000` at N=1, `late_episode`: the same envs timed again at those episode steps
(`value` stays the early-episode rate, the most expensive phase of an episode).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = ("env-steps/sec (whole node), 4-server LB env, batch 4k→512k at 1/2/4/8 MI355X")
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (8.0 TB/s spec)
ARRIVAL_RATE = 400.0   # flows/s per env (bench workload)
STEP_INTERVAL = 0.25   # simulated seconds per step
K = 128


def algorithmic_bytes(S: int, slots_per_env: float, inflight_per_env: float, paired: bool = False):
    """Bytes each kernel must move per env-step with the state layout of DESIGN.md §4.

    observe : read the 128 slot records ({fct, ts}: 8 B each, + the 4-B duration word of the
              duration plane when the handle has one -- paired = no plane, observe_pair_kernel)
              + hc + res_count per server, ep_step/ep_return read+write, obs 44 B/server,
              reward 4, done 1, ep outputs 12.
    dynamics: env header (8 x 4 B) and per-server hc/last_tc/res_count read+write, action 8 B and
              assign count 4 B per server, the reservoir slots actually written (8 B each, 12 with
              a duration plane; slots_per_env = lbsim_step_stats' popcount of the written-slot
              masks, measured on the timed steps), and the flows carried into the next step (8-B
              ring entry written at the end of the step and read at the start of the next:
              inflight_per_env).
    fused   : one launch does both, so both (the observe reads of freshly written records are
              algorithmic traffic even when L2 serves them).
    """
    rec = 8 if paired else 12
    obs = S * (K * rec + 8 + 44) + 12 + 12 + 4 + 1 + 12
    dyn = 2 * 32 + S * (2 * 12 + 8 + 4) + rec * slots_per_env + 16 * inflight_per_env
    return {"observe_kernel": obs, "dynamics_kernel": dyn, "fused_step_kernel": obs + dyn}


def phase_mismatch(workload, slots_per_env: float, name: str, tol: float = 0.10):
    """None if a committed counter file was collected on the same work as this run -- the
    reservoir slots written per env-step of its timed steps (the episode phase: early steps write
    more slots) within `tol` of this run's -- else the reason its counters do not apply."""
    if not workload or workload.get("slots_per_env_step") is None:
        return f"profiles/{name} does not record the slots per env-step its counters were taken at"
    ref = workload["slots_per_env_step"]
    if abs(ref - slots_per_env) > tol * max(slots_per_env, 1e-9):
        return (f"profiles/{name} was collected at {ref:.2f} reservoir slots per env-step "
                f"(steps {workload.get('bench_steps')}, warm-up {workload.get('bench_warmup')}); "
                f"this run wrote {slots_per_env:.2f}: another episode phase, counters not applied")
    return None


def valu_roofline(B: int, S: int, avg: dict, sigs: dict, slots_per_env: float = None):
    """The VALU side of each simulator kernel, from profiles/pmc_valu.json
    (tools/pmc_valu.py over rocprofv3 SQ counter passes of this workload, VALU issue costs measured
    by tools/ubench_valu.hip): VALU instructions per env-step and per class, the SIMD issue cycles
    they cost at the measured rates, and that issue time against this run's HIP-event kernel time
    (frac = issue_bound_ms / avg_launch_ms: 1.0 = the SIMDs never stop issuing VALU), plus the
    share of wave cycles parked on s_waitcnt / barriers (SQ_WAIT_ANY).  Counters are matched to
    the kernels that ran by their full template signature (sigs: lbsim_launch_names); a kernel
    whose signature the file does not hold gets {"pmc_kernel": None, "stale_reason": ...}, never
    another instantiation's counters.  None when the committed counters are for another shape."""
    path = os.path.join(ROOT, "profiles", "pmc_valu.json")
    if not os.path.exists(path):
        return None
    t = json.load(open(path))
    if t.get("batch") != B or t.get("servers") != S:
        return None
    out = {"source": "profiles/pmc_valu.json", "simds": t["simds"], "clock_hz": t["clock_hz"],
           "issue_costs_simd_cyc": t["ubench_simd_cyc_per_inst"], "workload": t.get("workload")}
    phase = phase_mismatch(t.get("workload"), slots_per_env, "pmc_valu.json") \
        if slots_per_env is not None else None
    for name in avg:
        if phase is not None:
            out[name] = {"pmc_kernel": None, "ran": sigs.get(name), "stale_reason": phase}
            continue
        full = sigs.get(name)
        rec = t["kernels"].get(full) if full else None
        if rec is None:
            out[name] = {"pmc_kernel": None, "ran": full,
                         "stale_reason": f"profiles/pmc_valu.json has no counters for {full!r} "
                                         f"(it holds {sorted(t['kernels'])})"}
            continue
        out[name] = {"pmc_kernel": full, "valu_per_env_step": rec["valu_per_env_step"],
                     "classes_per_env_step": rec["classes_per_env_step"],
                     "issue_bound_ms": rec["issue_bound_ms"], "avg_launch_ms": avg[name],
                     "frac": rec["issue_bound_ms"] / avg[name],
                     "wait_any_share": rec["wait_any_share"],
                     "active_valu_per_simd_quad": rec["active_valu_per_simd_quad"]}
    return out


def step_accounting(handle, lib, one_step, steps: int, replay=None):
    """Reservoir slots written and flows in flight per step (lbsim_step_stats after each step).
    replay = (twin factory, warm-up steps): the factory builds a second env from the same seeds
    and config with its own action generator (same seed), which walks the same trajectory bit for
    bit; its warm-up steps run uncounted, then exactly the timed steps are counted.  (A 0.5 GB
    state snapshot taken in the timed process slowed the timed steps by 1-3.5 %,
    profiles/r03/regress_r02_r03.txt.)  Else `steps` more steps of the same trajectory."""
    import torch
    twin = None
    if replay is not None:
        twin, one_step = replay[0]()
        handle = twin.handle
        for _ in range(replay[1]):
            one_step()
    st = (ctypes.c_int64 * 2)()
    slots = flows = 0
    for _ in range(steps):
        one_step()
        torch.cuda.synchronize()
        handle.check(lib.lbsim_step_stats(handle.h, st))
        slots += st[0]
        flows += st[1]
    if twin is not None:
        twin.close()
    return slots / steps, flows / steps


MFMA_F32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32, dense


def policy_flops(workload: str, S: int) -> float:
    """Algorithmic FLOPs per env-step of the fused policy kernel (multiply-adds x 2, unpadded).

    sac-gru: GRU (S*11 -> 128: three gates over input and hidden), fc1 128 -> 256, heads
             256 -> 2S (networks.py:19-146).
    qmix:    4 agents x [GRU (4k + 7S -> 64), fc1 64 -> 128, fc2 128 -> 128, fc3 128 -> 3]
             + mixer (state 4S + 10: four 64/32-wide first layers, 64 -> 128, 64 -> 32, 64 -> 1).
    """
    if workload == "sac-gru":
        i, h, f, a = S * 11, 128, 256, S
        return 2.0 * (i * 3 * h + h * 3 * h + h * f + f * 2 * a)
    k, ds = S // 4, 4 * S + 10
    obs = 4 * k + 7 * S
    agent = 2.0 * (obs * 192 + 64 * 192 + 64 * 128 + 128 * 128 + 128 * 3)
    mixer = 2.0 * (ds * (3 * 64 + 32) + 64 * 128 + 64 * 32 + 64 * 1)
    return 4 * agent + mixer


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None,
                    help="envs per GPU (default 65536; qmix 8192)")
    ap.add_argument("--servers", type=int, default=None,
                    help="servers per env (default 4; sac-gru 8; qmix 4 agents x 4)")
    ap.add_argument("--workload", choices=["rollout", "sac-gru", "qmix"], default="rollout",
                    help="rollout: random policy (configs[1] at the north-star batch); sac-gru: "
                         "problem-04 actor on GPU (configs[3]); qmix: problem-05 agents + "
                         "mixer on GPU (configs[4])")
    ap.add_argument("--seed", type=int, default=20260109)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--trace", default=None,
                    help="replay data/traces/<name>.npz (e.g. poisson_for_loop_rate_500: configs[2])")
    ap.add_argument("--policy", default="sed", help="sed | sed2 | lsq | lsq2 | alias")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dyn-mapping", default="auto", choices=["auto", "env", "server"],
                    help="dynamics kernel mapping: one lane per env / per server (same results)")
    ap.add_argument("--graph-steps", type=int, default=20,
                    help="steps captured per graph in the graph leg (one replay = that many steps: "
                         "a replay costs ~27 us besides its kernels -- torch's two RNG-offset fill "
                         "kernels and the launch -- so 20 steps amortise it to ~1.4 us per step, "
                         "profiles/r06l/)")
    ap.add_argument("--no-graph", action="store_true",
                    help="skip the graph leg (N=1: the same workload with --graph-steps steps captured in a "
                         "hipGraph and replayed, reported beside `value` as `graph`)")
    ap.add_argument("--async-groups", type=int, default=0,
                    help="rollout workload at N=1: after the headline, also time the same rollout "
                         "as this many env groups (B / groups envs each, global ids kept), each "
                         "stepped on its own HIP stream with no join between groups per step "
                         "(EnvPool-style async groups).  Off by default; reported beside `value`, "
                         "never as it")
    ap.add_argument("--prewarm-ms", type=float, default=200.0,
                    help="before the measured env is created, step a scratch env of the same "
                         "shape for at least this long (GPU clocks and caches ramp up); the "
                         "measured env's trajectory, warm-up and timed steps are unchanged.  "
                         "Reported as prewarm_ms; 0 disables")
    ap.add_argument("--autoreset-mode", choices=["same_step", "next_step"], default="same_step",
                    help="rollout workload: the env's auto-reset mode (same_step: SB3 / gym; "
                         "next_step: gymnasium >= 1.0's NEXT_STEP, the reset inside the step "
                         "launches -- the mode the graph leg always captures)")
    ap.add_argument("--graph-child", type=float, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--late-episode", default="",
                    help="rollout workload at N=1: after the headline measurement, keep stepping the "
                         "same envs and also time --steps steps from these episode steps (comma "
                         "list, e.g. 1000,5000; off by default so a profile of the default command "
                         "covers exactly the headline steps).  Reported beside `value`, never as it")
    return ap.parse_args()


def _cpu_info():
    """CPU model, affinity core count and the cgroup CPU quota (cpu.max) of this process."""
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return model or "host CPU", cores, quota


def cpu_baseline(args, seconds: float):
    """Oracle (C restatement, identical dynamics/features) on ALL of this process's cores
    (sched_getaffinity, one OpenMP thread each), bounded sample of the same workload: >= 64 envs
    per thread, about `seconds` of stepping.  Beside it, the reference's own CPU step
    (env.py simulation mode: MT19937 observations, dict round trip, reward; no flow dynamics),
    restated in marllb_amd.plumbing and timed here on one core, and the figure the survey
    recorded for the reference itself on a different host."""
    import numpy as np

    import oracle
    from marllb_amd.env import LoadBalanceEnv, make_config
    model, affinity, quota = _cpu_info()
    # every CPU this process may use: the affinity set, capped by the cgroup quota (on the GPU
    # box the affinity mask lists the whole machine, 256, but cpu.max grants 16; 256 threads on
    # 16 CPUs of quota run 4x slower than 16 threads: throttling, not the host's capability)
    threads = affinity if quota is None else max(1, min(affinity, int(quota + 0.999)))
    rng = np.random.default_rng(1)

    def timed(nb, S, secs, trace=None):
        """Oracle env-steps/s over nb envs (global ids 0..nb-1) x S servers for ~secs."""
        kw = {"trace": trace} if trace is not None else {}
        cfg = make_config(nb, S, seed=args.seed, env_id_offset=0, **kw)
        ora = oracle.OracleEnv(cfg, threads=threads, trace=trace)
        ora.reset()
        acts = [rng.integers(0, 3, (nb, S)).astype(np.int64) for _ in range(8)]
        ora.step(acts[0])  # warm caches / thread pool
        n, t0 = 0, time.perf_counter()
        while True:
            ora.step(acts[n % len(acts)])
            n += 1
            el = time.perf_counter() - t0
            if el >= secs and n >= 3:
                break
        ora.close()
        return nb * n / el, n, el

    nb = max(2048, 64 * threads)
    rate, n, el = timed(nb, args.servers, seconds)
    # BASELINE.md §3's two CPU points: configs[1] 4096 x 4 (every env) and configs[2] 65536 x 8
    # trace replay (a sample of its envs), each ~seconds/2
    from marllb_amd import trace as lbtrace
    points = []
    for name, nb_p, S_p, tr in (("configs[1] 4096 x 4, random policy, all 4096 envs", 4096, 4, None),
                                ("configs[2] 65536 x 8, rate_500 trace replay, envs 0-4095 of "
                                 "65536 sampled", 4096, 8, lbtrace.builtin())):
        r_p, n_p, el_p = timed(nb_p, S_p, seconds / 2, tr)
        points.append({"config": name, "value": r_p, "unit": "env-steps/s", "cores": threads,
                       "kind": "port", "steps": n_p, "seconds": el_p})
    # the reference's CPU plumbing step (configs[0], 1 x S, step_interval 0), one core
    pe = LoadBalanceEnv(num_servers=args.servers, step_interval=0.0, seed=0,
                        reference_plumbing=True)
    pe.reset()
    pa = [rng.integers(0, 3, args.servers) for _ in range(64)]
    m, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < 2.0:
        pe.step(pa[m % 64])
        m += 1
    pel = time.perf_counter() - t1
    return {"value": rate, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "baseline_points": points,
            "cpu_model": model, "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "sample": f"{nb} of the {args.batch} envs (global ids 0-{nb - 1}), S={args.servers}, "
                      f"{n} random-policy steps, {el:.1f} s, oracle/lbsim_oracle.c "
                      f"(OpenMP, {threads} threads = every CPU available: sched_getaffinity "
                      f"{affinity}, cgroup quota {quota}) on {model}",
            "reference_plumbing": {
                "value": m / pel, "unit": "env-steps/s/core", "cores": 1, "kind": "port",
                "what": "the reference's own LoadBalanceEnv.step in simulation mode (random "
                        "observations, no flow dynamics, step_interval=0), restated byte-exact "
                        "in marllb_amd/plumbing.py, timed here",
                "survey_recorded": {"value": 8164.0, "unit": "env-steps/s/core",
                                    "host": "different host: survey container, Intel Xeon "
                                            "8 vCPU, reference Python run in place "
                                            "(SURVEY.md §6, BASELINE.md §2)"}}}


def async_groups(args, dev, shard, B, S, common, groups):
    """The headline rollout as `groups` env groups of B / groups envs (global ids kept, so the
    same envs), each stepped on its own HIP stream with its own random-action generator and no
    join between groups inside a step: a group's next dynamics launch can start while another
    group's observe is running, filling the SIMDs that the latency-bound dynamics kernel's tail
    leaves idle (one step = every group advances one env step; warmup and timing as the headline;
    profiles/r02_round2c/stream_split_*.jsonl).  A different calling pattern from one batched
    step(), so it is reported beside `value`, never as it."""
    import torch
    from marllb_amd.env import VecLoadBalanceEnv
    b = B // groups
    streams = [torch.cuda.Stream(dev) for _ in range(groups)]
    envs, gens = [], []
    for i in range(groups):
        kw = dict(common)
        kw["env_id_offset"] = shard.env_id_offset + i * b
        with torch.cuda.stream(streams[i]):
            e = VecLoadBalanceEnv(b, S, max_steps=10000, **kw)
            e.reset()
            g = torch.Generator(device=dev)
            g.manual_seed(args.seed + 1000 + i)
        envs.append(e)
        gens.append(g)

    def step_all():
        for i in range(groups):
            with torch.cuda.stream(streams[i]):
                a = torch.randint(0, 3, (b, S), device=dev, dtype=torch.int64, generator=gens[i])
                envs[i].step(a)

    for _ in range(args.warmup):
        step_all()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step_all()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    for e in envs:
        e.close()
    return {"groups": groups, "envs_per_group": b, "value": groups * b * args.steps / el,
            "unit": "env-steps/s", "ms_per_step": el / args.steps * 1e3,
            "streams": "one HIP stream per group, no cross-group join per step"}


def graph_leg(args, dev, shard, B, S, common, kernel_ms):
    """The same workload with k = --graph-steps steps captured into one torch.cuda.CUDAGraph (hipGraph) and
    replayed: a fresh env in graph_mode with static buffers -- the random-policy rollout with
    next-step auto-reset (the resets run inside the step launches, so the captured step is the
    eager step's two launches and nothing else), the policy rollouts with the same-step masked
    auto-reset launched every step -- the random policy's torch.randint (default generator,
    graph-safe) or the fused policy kernel (Philox step counter on the device) inside the graph.  Same kernels and work per step
    as the eager headline, without the per-launch host path; `gap_ms_per_step` = replayed
    ms/step - the eager kernels' HIP-event averages = what the launches between the kernels
    still cost.  Reported beside `value`, never as it."""
    import torch
    from marllb_amd.env import VecLoadBalanceEnv
    common = dict(common, graph_mode=True)
    common.pop("autoreset_mode", None)
    autoreset = "same_step"
    k = max(1, args.graph_steps)  # steps per captured graph (one replay = k steps)
    if args.workload == "rollout":
        autoreset = "next_step"
        env = VecLoadBalanceEnv(B, S, max_steps=10000, autoreset_mode=autoreset, **common)
        env.reset()
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):
                env.step(torch.randint(0, 3, (B, S), device=dev, dtype=torch.int64))
        torch.cuda.current_stream(dev).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(k):
                env.step(torch.randint(0, 3, (B, S), device=dev, dtype=torch.int64))
    elif args.workload == "sac-gru":
        from marllb_amd.rollout import SACGRURollout
        env = VecLoadBalanceEnv(B, S, action_type="continuous", max_steps=10000, **common)
        g = SACGRURollout(env, seed=args.seed + shard.rank).capture(steps=k)
    else:
        from marllb_amd.multi_agent import VecMultiAgentLoadBalanceEnv
        from marllb_amd.rollout import QMIXRollout
        env = VecMultiAgentLoadBalanceEnv(B, 4, S // 4, action_type="discrete", max_steps=100,
                                          **common)
        g = QMIXRollout(env, seed=args.seed + shard.rank).capture(steps=k)
    # the kernels the captured step launches (next-step handles: the kModeStepNR dynamics), so
    # gap_ms_per_step is read against the right eager kernels
    from marllb_amd import _lib
    h = env.handle if hasattr(env, "handle") else getattr(getattr(env, "vec", None), "handle", None)
    ran = _lib.launch_names(h, 0) if h is not None else {}
    reps = max(1, -(-args.steps // k))  # replays covering at least --steps steps
    for _ in range(max(1, -(-args.warmup // k))):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    env.close()
    n = reps * k
    ms = el / n * 1e3
    return {"value": B * n / el, "unit": "env-steps/s", "ms_per_step": ms, "steps": n,
            "kernels_ms_per_step": kernel_ms, "gap_ms_per_step": ms - kernel_ms,
            "form": f"{k} steps captured in one torch.cuda.CUDAGraph, replayed",
            "steps_per_graph": k, "autoreset": autoreset, "kernels": ran,
            "note": "kernels_ms_per_step are the eager leg's HIP-event averages; the graph leg "
                    "runs the kernels in `kernels` (compare with the eager line's signatures when "
                    "the auto-reset modes differ)"}


def graph_leg_child(args, kernel_ms, timeout_s: float = 420.0):
    """Runs graph_leg in a fresh child process (this script with --graph-child) and returns its
    dict: a fault or abort inside the HIP runtime during graph capture / replay ends the child, not
    the headline process, whose JSON line is then printed with graph = {"error": ...} (VERDICT r05
    item 6: a runtime abort there used to lose the headline).  The child starts as a new program
    (fork + exec of python by subprocess, no exec of this process) and initialises its own GPU
    context; it builds the same workload from the same arguments."""
    import subprocess
    argv = [sys.executable, os.path.abspath(__file__)] + [a for a in sys.argv[1:]] + \
        ["--graph-child", repr(kernel_ms), "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK")}
    try:
        r = subprocess.run(argv, env=env, capture_output=True, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return {"error": f"graph-leg child timed out after {timeout_s:.0f} s"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        tail = " | ".join(r.stderr.strip().splitlines()[-4:])
        return {"error": f"graph-leg child exited {r.returncode}: {tail}"}
    res = json.loads(lines[-1])
    res["process"] = "child (fresh process and GPU context; the headline process never captures)"
    return res


def late_episode(args, env, handle, lib, one_step, rate, B, S, done_steps):
    """The same rollout later in its episodes (max_steps 10000, the reference default): every
    reservoir is full and most servers' reservoirs take no new sample in a step (Algorithm R
    acceptance 128 / count), so observe reuses most feature rows.  The headline
    `value` is the early-episode rate (the most expensive phase); this reports where the episode
    spends most of its steps.  Untimed stepping to each start point, then --steps timed steps."""
    import torch
    res = []
    step = done_steps
    for target in sorted(int(x) for x in args.late_episode.split(",") if x.strip()):
        while step < target:
            one_step()
            step += 1
        torch.cuda.synchronize()
        handle.check(lib.lbsim_profile_begin(handle.h, 4 * args.steps + 8))
        t0 = time.perf_counter()
        for _ in range(args.steps):
            one_step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        NC = 5
        ms = (ctypes.c_double * NC)()
        cnt = (ctypes.c_int64 * NC)()
        handle.check(lib.lbsim_profile_end_ex(handle.h, ms, cnt, NC))
        step += args.steps
        names = {0: "dynamics", 1: "observe", 4: "fused_step"}
        res.append({"episode_step": target, "value": B * args.steps / el, "unit": "env-steps/s",
                    "ms_per_step": el / args.steps * 1e3,
                    "kernel_avg_ms": {names[i]: ms[i] / cnt[i] for i in names if cnt[i] > 0}})
    return res


def prewarm_scratch(args, dev, B, S, common):
    """Step a scratch env of the measured shape (its own seed, destroyed afterwards) for at least
    --prewarm-ms of wall time, so the timed region does not start on an idle GPU's clocks.  The
    measured env is created after it: its trajectory, W warm-up and K timed steps are exactly
    those of a run without the pre-warm (the slots written per step depend on the episode
    phase, so pre-warming on the measured env itself would change the timed work)."""
    import torch
    from marllb_amd.env import VecLoadBalanceEnv
    if args.prewarm_ms <= 0:
        return None
    kw = dict(common, seed=args.seed ^ 0x5A5A5A5A)
    if args.workload == "sac-gru":
        kw["action_type"] = "continuous"
    env = VecLoadBalanceEnv(B, S, max_steps=10000, **kw)
    env.reset()
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed + 7)
    continuous = args.workload == "sac-gru"
    n, t0 = 0, time.perf_counter()
    while True:
        if continuous:
            a = torch.rand((B, S), device=dev, generator=gen) * 2.0
        else:
            a = torch.randint(0, 3, (B, S), device=dev, dtype=torch.int64, generator=gen)
        env.step(a)
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize()
            if (time.perf_counter() - t0) * 1e3 >= args.prewarm_ms:
                break
    el = (time.perf_counter() - t0) * 1e3
    env.close()
    torch.cuda.synchronize()
    return {"prewarm_ms": el, "steps": n,
            "form": "a scratch env of the same shape (own seed), created, stepped and destroyed "
                    "before the measured env exists; not part of W or K"}


def spawn_ranks(args) -> int:
    """`bench.py --gpus N` without torchrun: start N rank processes of this script (one per GPU,
    the torchrun environment contract: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), before this
    parent touches the GPU; only rank 0 prints the JSON line.  Returns the worst exit code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = {**os.environ, "RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(args.gpus),
               "LOCAL_WORLD_SIZE": str(args.gpus), "GROUP_RANK": "0",
               "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)}
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or code
                for q in live:  # one rank failed: the others would wait in a collective
                    q.terminate()
        time.sleep(0.2)
    return rc


def main():
    args = parse()
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(spawn_ranks(args))
    import torch
    import torch.distributed as dist

    from marllb_amd import _lib
    from marllb_amd import dist as lbdist
    from marllb_amd.env import VecLoadBalanceEnv

    if args.batch is None:
        args.batch = 8192 if args.workload == "qmix" else 65536
    if args.servers is None:
        args.servers = {"rollout": 4, "sac-gru": 8, "qmix": 16}[args.workload]
    shard = lbdist.from_env(args.batch)
    world, rank = shard.world, shard.rank
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # one process per GPU; LBSIM_DIST_BACKEND=gloo rehearses several ranks on fewer GPUs
    backend = os.environ.get("LBSIM_DIST_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # a process group whenever a launcher gave this process a rank (torchrun's contract), N = 1
    # included: the timing barrier and the max / gather of the elapsed times then run as RCCL
    # collectives on the GPU at every N (tests/test_dist.py::test_bench_torchrun_rccl_world1)
    dist_on = world > 1 or ("RANK" in os.environ and args.graph_child is None)
    if dist_on:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    B, S = args.batch, args.servers
    tr = None
    if args.trace:
        from marllb_amd import trace
        tr = trace.builtin(args.trace)
    common = dict(device=dev, seed=args.seed, env_id_offset=shard.env_id_offset, autoreset=True,
                  assign_policy=args.policy, trace=tr, dyn_mapping=args.dyn_mapping)
    if args.workload == "rollout":
        common["autoreset_mode"] = args.autoreset_mode
    if args.graph_child is not None:  # the graph leg alone, in its own process (graph_leg_child)
        # the same pre-warm as the eager leg (a scratch env, --prewarm-ms): without it the child's
        # 20 replayed steps ran on a cold GPU's clocks (r06f: 0.283 ms/step against 0.262 eager
        # on the same next-step kernels)
        pw = prewarm_scratch(args, dev, B, S, common)
        res = graph_leg(args, dev, shard, B, S, dict(common), args.graph_child)
        res["prewarm"] = pw
        print(json.dumps(res), flush=True)
        return
    prewarm = prewarm_scratch(args, dev, B, S, common)
    torch.manual_seed(args.seed)  # network init (random weights of the reference architecture)
    if args.workload == "rollout":
        env = VecLoadBalanceEnv(B, S, max_steps=10000, **common)
        env.reset()
        handle = env.handle
        gen = torch.Generator(device=dev)
        gen.manual_seed(args.seed + rank)

        def one_step():
            a = torch.randint(0, 3, (B, S), device=dev, dtype=torch.int64, generator=gen)
            env.step(a)
    elif args.workload == "sac-gru":
        from marllb_amd.rollout import SACGRURollout
        env = VecLoadBalanceEnv(B, S, action_type="continuous", max_steps=10000, **common)
        ro = SACGRURollout(env, seed=args.seed + rank)
        handle = env.handle

        def one_step():
            ro.step()
    else:
        from marllb_amd.multi_agent import VecMultiAgentLoadBalanceEnv
        from marllb_amd.rollout import QMIXRollout
        if S % 4:
            raise SystemExit("qmix workload: servers must be 4 agents x k")
        env = VecMultiAgentLoadBalanceEnv(B, 4, S // 4, action_type="discrete", max_steps=100,
                                          **common)
        ro = QMIXRollout(env, seed=args.seed + rank)
        handle = env.vec.handle

        def one_step():
            ro.step()

    replay = None
    if args.workload == "rollout" and rank == 0:  # exact accounting replay of warm-up + timed steps

        def twin():
            e2 = VecLoadBalanceEnv(B, S, max_steps=10000, **common)
            e2.reset()
            g2 = torch.Generator(device=dev)
            g2.manual_seed(args.seed + rank)

            def step2():
                e2.step(torch.randint(0, 3, (B, S), device=dev, dtype=torch.int64, generator=g2))
            return e2, step2
        replay = (twin, args.warmup)
    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    lib = _lib.load()
    from marllb_amd import policies
    if args.workload != "rollout":  # HIP events around each fused policy launch
        policies.profile_events = []
    handle.check(lib.lbsim_profile_begin(handle.h, 4 * args.steps + 8))
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist_on:
        dist.barrier()
    NC = _lib.PROFILE_CLASSES
    ms = (ctypes.c_double * NC)()
    cnt = (ctypes.c_int64 * NC)()
    handle.check(lib.lbsim_profile_end_ex(handle.h, ms, cnt, NC))
    pol_events, policies.profile_events = policies.profile_events, None
    cdev = dev if backend == "nccl" else None
    elapsed = lbdist.max_over_ranks(t1 - t0, cdev)
    per_rank = lbdist.gather_over_ranks(t1 - t0, cdev)
    # the graph leg right after the timed region (before the accounting replay and everything
    # else), so both legs run on the GPU in a similar state: sustained load lowers the kernels'
    # speed over the following seconds (profiles/r05k/).  In a child process: nothing the capture
    # or the replays do can abort this one (graph_leg_child).
    graph_res = None
    if world == 1 and not args.no_graph:
        kms = sum(ms[i] / cnt[i] for i in (0, 1, 4) if cnt[i] > 0)
        if pol_events:
            kms += sum(a.elapsed_time(b) for a, b in pol_events) / len(pol_events)
        graph_res = graph_leg_child(args, kms)

    if rank == 0:
        value = lbdist.throughput(shard, args.steps, elapsed)
        # a step is one fused_step_kernel launch (opt-in) or a dynamics launch -- dynamics_group_kernel
        # (one lane per server), dynamics_wave_kernel (one wave per env, small S <= 4 batches) or
        # dynamics_kernel (one lane per env, --dyn-mapping env) -- then observe_kernel;
        # lbsim_profile times each class
        dyn = ("dynamics_kernel", "dynamics_group_kernel",
               "dynamics_wave_kernel")[lib.lbsim_dynamics_kernel(handle.h)]
        # the template signature of each kernel the step launched (lbsim_launch_names), the key
        # of the committed PMC counter files; the one-launch step's kernel named from it
        ran = _lib.launch_names(handle, 0) if hasattr(lib, "lbsim_launch_names") else {}
        fused = ran.get(4, "").split("<")[0] or (
            "step_wave_kernel" if dyn == "dynamics_wave_kernel" else "fused_step_kernel")
        obs_name = ran.get(1, "observe_kernel").split("<")[0]
        names = {0: dyn, 1: obs_name, 4: fused}
        avg = {names[i]: ms[i] / cnt[i] for i in names if cnt[i] > 0}
        rate = tr.rate if tr is not None else ARRIVAL_RATE
        slots, inflight = step_accounting(handle, lib, one_step, args.steps, replay)
        abytes = algorithmic_bytes(S, slots / B, inflight / B,
                                   paired=True)  # duration "age", lost-FIN off: no plane
        abytes[obs_name] = abytes.pop("observe_kernel")
        abytes[dyn] = abytes.pop("dynamics_kernel")
        abytes[fused] = abytes.pop("fused_step_kernel")
        per_kernel = {}
        for k in avg:
            ab_k = abytes[k] * B
            ach = ab_k / (avg[k] * 1e-3) / 1e9
            per_kernel[k] = {"avg_launch_ms": avg[k], "algorithmic_bytes_per_launch": ab_k,
                             "achieved_GBps": ach, "frac": ach / HBM_PEAK_GBS}
        sigs = {names[c]: sig for c, sig in ran.items() if c in names}
        for k in per_kernel:
            per_kernel[k]["signature"] = sigs.get(k)
        dom = max(avg, key=avg.get)
        ab = abytes[dom] * B
        achieved = ab / (avg[dom] * 1e-3) / 1e9
        valu = valu_roofline(B, S, avg, sigs, slots / B)
        traffic, traffic_note, traffic_workload = None, None, None
        tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(tfile):
            t = json.load(open(tfile))
            held = t.get("bytes_per_launch", {})
            traffic_workload = t.get("workload")
            if t.get("batch") != B or t.get("servers") != S:
                traffic_note = f"profiles/pmc_traffic.json is for {t.get('batch')} x {t.get('servers')}"
            elif sigs.get(dom) not in held:
                traffic_note = (f"profiles/pmc_traffic.json has no counters for {sigs.get(dom)!r} "
                                f"(it holds {sorted(held)})")
            else:
                traffic_note = phase_mismatch(traffic_workload, slots / B, "pmc_traffic.json")
                if traffic_note is None:
                    traffic = held[sigs[dom]]
        out = {
            "metric": METRIC, "value": value, "unit": "env-steps/s",
            "n_gpus": dist.get_world_size() if world > 1 else 1,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            # every rank's timed-region wall time (value uses the max): imbalance shows here
            "ranks": {"world_size": world, "backend": backend if dist_on else None,
                      "elapsed_s": per_rank, "elapsed_min_s": min(per_rank),
                      "elapsed_max_s": elapsed},
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32/int32 (f64 reward)",
            "data": ("synthetic: Philox4x32-10 Poisson arrivals lambda=400/s, Exp(1) work, "
                     "mu=lambda/(0.8 S) per server, random discrete policy") if tr is None else
                    (f"trace replay {tr.name} ({tr.rows} rows, {tr.rate:.1f}/s; per-env offset "
                     "gid*7919), mu=rate/(0.8 S), random discrete policy"),
            "config": {"workload": (f"LB env random-policy rollout, {S} servers (BASELINE "
                                    "configs[1] rollout at the north-star batch)" if S == 4
                                    and B == 65536 else f"LB env random-policy rollout, {B} x "
                                    f"{S} (BASELINE configs[1] shape family)") if tr is None else
                                   f"LB env trace replay, {S} servers (BASELINE configs[2])",
                       "assign_policy": args.policy,
                       "envs_per_gpu": B, "servers": S, "global_batch": world * B,
                       "step_interval_s": 0.25, "autoreset": True,
                       "autoreset_mode": args.autoreset_mode if args.workload == "rollout"
                       else "same_step",
                       "parallelism": f"env-shard x{world}", "dyn_mapping": args.dyn_mapping},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_source": "profiles/pmc_traffic.json"
                         if traffic is not None else None, "stale_reason": traffic_note,
                         "traffic_workload": traffic_workload,
                         "signature": sigs.get(dom), "algorithmic_bytes_per_launch": ab,
                         "avg_launch_ms": avg[dom],
                         "kernel_avg_ms": avg, "kernels": per_kernel, "valu": valu,
                         # the two simulator kernels take about equal time: `kernel` is the longer
                         # one this run; the dynamics kernel moves few bytes by construction (an
                         # event loop, latency-bound: see `valu`), observe is the HBM-heavy one
                         "hbm_heavy_kernel": (max(per_kernel, key=lambda k: per_kernel[k]
                                                  ["algorithmic_bytes_per_launch"])
                                              if per_kernel else None),
                         "accounting": {"reservoir_slots_written_per_env_step": slots / B,
                                        "flows_in_flight_per_env": inflight / B,
                                        "basis": "lbsim_step_stats after each step of an exact "
                                                 "replay of the timed steps" if replay else
                                                 "lbsim_step_stats over as many further steps"}},
        }
        out["prewarm"] = prewarm
        if args.workload != "rollout":
            out["config"]["workload"] = {
                "sac-gru": f"problem-04 SAC-GRU actor (GRU {S * 11}->128, fc 128->256, heads "
                           f"256->{S}) sampling continuous weights on the GPU each step, "
                           f"{S} servers (BASELINE configs[3] per GPU)",
                "qmix": f"problem-05 QMIX: 4 agents x {S // 4} servers, per-agent GRU "
                        f"Q-networks (obs {4 * (S // 4) + 7 * S}) epsilon-greedy + mixing network "
                        f"(state {4 * S + 10}) on the GPU each step (BASELINE configs[4] per GPU)"}[
                            args.workload]
            out["data"] = out["data"].replace("random discrete policy",
                                              "random-init network policy")
            out["policy_ms_per_step"] = out["ms_per_step"] - sum(avg.values())
            out["config"]["fused_policy_tile"] = os.environ.get("LBSIM_FUSED_MT", "auto")
            if pol_events:
                pms = sum(a.elapsed_time(b) for a, b in pol_events) / len(pol_events)
                fl = policy_flops(args.workload, S) * B
                tf = fl / (pms * 1e-3) / 1e12
                name = {"sac-gru": "sac_actor_kernel", "qmix": "qmix_policy_kernel"}[args.workload]
                out["roofline"]["kernels"][name] = {
                    "bound": "mfma", "avg_launch_ms": pms, "flops_per_launch": fl,
                    "achieved_TFLOPs": tf, "peak_TFLOPs": MFMA_F32_PEAK_TFLOPS,
                    "frac": tf / MFMA_F32_PEAK_TFLOPS}
                # host + torch work between the launches (<= 10 us)
                out["policy_glue_ms_per_step"] = out["policy_ms_per_step"] - pms
        if graph_res is not None:
            out["graph"] = graph_res
        if world == 1 and args.workload == "rollout" and args.late_episode:
            out["late_episode"] = late_episode(args, env, handle, lib, one_step, rate, B, S,
                                               args.warmup + args.steps)
        if world == 1 and args.workload == "rollout" and args.async_groups > 1:
            out["async_groups"] = async_groups(args, dev, shard, B, S, common, args.async_groups)
        if world == 1 and not args.no_cpu_baseline and args.workload == "rollout":
            out["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    env.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
