"""Benchmark: Fisher-z CI tests/s + PC skeleton wall-time, synthetic Gaussian SEM
(BASELINE.json config 5: 2000 vars x 10 000 samples, max conditioning depth 4, alpha 0.05).

One step = one full stable-PC skeleton on data already resident in HBM: K1 correlation
(fp64 MFMA) + every depth 0..4 (work-list build, CI-test kernel, exact path, level barrier);
on one GPU both run in one C call (pcg_pc_skeleton, stream-ordered, no host round trip).
N=1: one GPU. N>1 (torchrun): the same skeleton edge-sharded across ranks, removal flags
merged with an RCCL all-reduce at every level barrier (strong scaling of one fixed graph).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Fisher-z CI tests/sec + PC skeleton wall-time (2000 vars), 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0        # MI355X spec (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6      # MI355X fp64 (vector = matrix) spec


def bytes_per_test(d: int) -> int:
    """unique sub-matrix entries + indices + p-value out."""
    return 8 * (d + 2) * (d + 3) // 2 + 4 * (d + 2) + 8


def _latest(pattern: str):
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    return files[-1] if files else None


def _pmc(kernel: str):
    """Per-dispatch PMC counters of ``kernel`` (rocprof name, template args kept) from the latest
    committed rocprofv3 passes over this same bench command (profiles/r*_pmc_summary.json)."""
    f = _latest("r*_pmc_summary.json")
    if not f:
        return {}, None
    ctr = json.load(open(f)).get(kernel, {})
    return {k: v["per_dispatch_mean"] for k, v in ctr.items()}, os.path.basename(f)


def _issue_model(kernel: str):
    """The committed VALU issue-cost model of ``kernel`` (tools/roofline_model.py): the kernel's
    per-dispatch VALU instructions by PMC class x the measured cycles of each class's opcodes
    (profiles/r03_issue_cost.json, split in the proportions of the kernel's own ISA)."""
    f = _latest("r*_roofline_model.json")
    if not f:
        return None, None
    m = json.load(open(f))
    return (m if m.get("kernel") == kernel else None), os.path.basename(f)


# The guide's VALU issue cost of one wave64 instruction on a SIMD-32 with other waves to interleave
# (MI355X_MICROARCH.md:54,473: a non-packed FP32 / INT32 VALU occupies the SIMD 2 cycles; packed
# FP32 and FP64 4; transcendentals 8)
TRANSCENDENTAL = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")


def guide_cycles(op: str) -> float:
    if op.startswith(TRANSCENDENTAL):
        return 8.0
    if op.startswith("v_pk_") or "f64" in op or op.startswith(("v_lshl_add_u64", "v_mad_u64", "v_mad_i64")):
        return 4.0
    return 2.0


def guide_issue_cycles(model: dict) -> float:
    """SIMD-cycles of the kernel's dynamic VALU instruction mix at the guide's issue costs: every
    PMC class count of every region split over its opcodes in the proportions of the region's own
    ISA (as tools/roofline_model.py splits them), each opcode at guide_cycles."""
    tot = 0.0
    for reg in model["regions"].values():
        for cls in reg["classes"].values():
            ops = cls.get("isa_static") or {}
            n_static = sum(ops.values())
            if not n_static:
                tot += 2.0 * cls["dynamic"]
                continue
            tot += cls["dynamic"] * sum(c * guide_cycles(op) for op, c in ops.items()) / n_static
    return tot


def roofline_of(kernel: str, tests: int, d: int, k_ms: float) -> dict:
    """Roofline of the dominant CI-test kernel.

    Binding resource: VALU issue. The kernel stages each node's correlation block in LDS, so
    its HBM traffic (PMC) is far below SURVEY §8(d)'s per-test byte model and HBM is not what
    binds. achieved = the SIMD-cycles its VALU instructions need to issue at the GUIDE's rates,
    per launch ÷ the live kernel time; peak = 1024 SIMDs × 2.4 GHz; frac = achieved / peak.

    The instruction mix is the committed model's (profiles/r*_roofline_model.json,
    tools/roofline_model.py): the PMC class counters of this kernel on this bench command
    (SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_{F32,F64}, _INT32, _INT64, _CVT, SQ_INSTS_VALU for the
    rest), each class split over its opcodes in the proportions of the kernel's ISA. Costed at
    the guide's issue cycles (guide_cycles: 2 non-packed, 4 packed / fp64, 8 transcendental) that
    gives `frac`; costed at the cycles tools/micro/issue_cost.hip MEASURED for those opcodes at the
    kernel's occupancy (VOP3 v_fma_f32 with its sources in one VGPR bank 4.56, packed 4.6 —
    profiles/r03_issue_cost.json) it gives `frac_model`, with that model's bounds."""
    peak_gcyc = 1024 * 2.4   # G SIMD-cycles/s
    line = {"bound": "valu", "unit": "G SIMD-cycles/s (VALU issue at the guide's rates)", "peak": peak_gcyc,
            "achieved": None, "frac": None, "traffic": None, "kernel": kernel, "kernel_ms": k_ms}
    alg = tests * bytes_per_test(d)
    sec = {"hbm_contract_bytes_per_test": bytes_per_test(d),
           "hbm_contract_gbs": alg / (k_ms / 1e3) / 1e9 if k_ms > 0 else None,
           "note": "SURVEY 8(d) per-test byte model; operands are LDS-resident, so it is not a traffic figure"}
    model, msrc = _issue_model(kernel)
    line["model_source"] = msrc
    if k_ms > 0 and model:
        gcyc = guide_issue_cycles(model)
        line["achieved"] = gcyc / (k_ms / 1e3) / 1e9
        line["frac"] = line["achieved"] / peak_gcyc
        line["guide_issue_cycles_per_launch"] = gcyc
        cyc = float(model["valu_issue_cycles"])
        lo, hi = (float(v) for v in model["valu_issue_cycles_bounds"])
        line["frac_model"] = cyc / (k_ms / 1e3) / 1e9 / peak_gcyc
        line["frac_model_bounds"] = [lo / (k_ms / 1e3) / 1e9 / peak_gcyc, hi / (k_ms / 1e3) / 1e9 / peak_gcyc]
        line["valu_issue_cycles_per_launch"] = cyc
        line["valu_instructions_per_launch"] = model["valu_instructions"]
        line["mean_cycles_per_valu"] = model["mean_cycles_per_valu"]
        sec["valu_instr_per_64_tests"] = model["valu_instructions"] / (tests / 64.0) if tests else None
    ctr, src = _pmc(kernel)
    line["pmc_source"] = src
    if k_ms > 0 and "FETCH_SIZE" in ctr and "WRITE_SIZE" in ctr:
        # FETCH_SIZE counts KiB with gfx950's wide reads at half weight (MI355X_MICROARCH.md HBM
        # section): x2; WRITE_SIZE KiB as is
        traffic = ctr["FETCH_SIZE"] * 1024.0 * 2.0 + ctr["WRITE_SIZE"] * 1024.0
        line["traffic"] = traffic
        sec["hbm_measured_gbs"] = traffic / (k_ms / 1e3) / 1e9
        sec["hbm_measured_frac"] = sec["hbm_measured_gbs"] / HBM_PEAK_GBS
    line["secondary"] = sec
    return line


K1_TILE = 64                  # corr.hip tile (both paths)
K1_DIGITS = 9                 # corr.hip K1_DIG: int8 digits per value
I8_PEAK_TOPS = 5000.0         # MI355X dense int8 MFMA (2x the dense BF16 rate; MI355X_MICROARCH.md)
MFMA_F64_MEASURED_TFLOPS = 47.9   # v_mfma_f64_16x16x4_f64 at 4 waves/SIMD, tools/micro/mfma_f64.hip (profiles/r02_mfma_f64.log)


CRT_MODULI = (256, 255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 217, 211, 199, 197, 193, 191, 181, 179, 173,
              167, 163, 157, 151)     # corr.hip kCrtModuli
CRT_TILE = 256


def k1_crt_moduli(n: int, N: int, tune: dict):
    """(k, b) of corr.hip's crt_plan, or None when K1 takes the digit / fp64 path: the fewest
    moduli whose product M leaves b >= PCG_TUNE_K1_CRT_BITS bits per value with M > 2 N 4^b."""
    if not tune["K1_I8"] or not tune["K1_CRT"] or n < tune["K1_CRT_MINN"]:
        return None
    bmin = tune["K1_CRT_BITS"]
    lm = 0.0
    for k, m in enumerate(CRT_MODULI, 1):
        lm += math.log2(m)
        b = math.floor((lm - math.log2(N) - 1.0 - 0.01) / 2.0)
        if b >= bmin:
            return k, min(b, 63)
    return None


def k1_roofline(n: int, N: int, corr_ms: float, tune: dict) -> dict:
    """K1 (np.corrcoef). Default path for n >= 256 (corr.hip, CRT): the centred X truncated to
    b-bit integers, k residue planes, the Gram as k exact int8 GEMMs of the upper-triangle
    256-square tiles on v_mfma_i32_32x32x32_i8, rebuilt by the Chinese remainder theorem;
    executed int8 ops = k x 2 x T(T+1)/2 x 256^2 x N_pad. Below n = 256: 9 digit planes and 45
    GEMMs of 64-square tiles. The fp64 path (PCG_K1_I8=0) runs v_mfma_f64_16x16x4_f64 on 64-square
    tiles. Either way the algorithmic work is 2 N n^2 (reported as achieved_algorithmic, TFLOP/s)."""
    i8 = bool(tune["K1_I8"])
    crt = k1_crt_moduli(n, N, tune)
    npad = (N + 63) // 64 * 64
    line = {"bound": "mfma", "ms": corr_ms, "path": "int8 CRT" if crt else ("int8 digits" if i8 else "fp64"),
            "achieved_algorithmic_tflops": 2.0 * N * n * n / (corr_ms / 1e3) / 1e12,
            "what": "pcg_corr end to end (column stats, residue / digit planes, split-K GEMM, rebuild, normalisation)"}
    if crt:
        k, b = crt
        T = (n + CRT_TILE - 1) // CRT_TILE
        ops = k * 2.0 * (T * (T + 1) // 2) * CRT_TILE * CRT_TILE * npad
        ex = ops / (corr_ms / 1e3) / 1e12
        line.update({"moduli": k, "bits": b, "unit": "TOP/s (int8)", "peak": I8_PEAK_TOPS, "achieved_executed": ex,
                     "frac": ex / I8_PEAK_TOPS})
        return line
    T = (n + K1_TILE - 1) // K1_TILE
    tiles = T * (T + 1) // 2
    if i8:
        ops = K1_DIGITS * (K1_DIGITS + 1) // 2 * 2.0 * tiles * K1_TILE * K1_TILE * npad
        ex = ops / (corr_ms / 1e3) / 1e12
        line.update({"unit": "TOP/s (int8)", "peak": I8_PEAK_TOPS, "achieved_executed": ex, "frac": ex / I8_PEAK_TOPS})
    else:
        mfma_flop = tiles * K1_TILE * K1_TILE * 2.0 * N
        ex = mfma_flop / (corr_ms / 1e3) / 1e12
        line.update({"unit": "TFLOP/s", "peak": FP64_PEAK_TFLOPS, "achieved_executed": ex,
                     "frac": ex / FP64_PEAK_TFLOPS,
                     "frac_of_measured_instruction_ceiling": ex / MFMA_F64_MEASURED_TFLOPS})
    return line


def dominant_kernel(d: int, full_p: bool, screen_mask: int = -1) -> str:
    """Name (as rocprofv3 prints it, template args kept) of the CI-test kernel that runs
    depth ``d`` for nodes of degree <= 64 — the host dispatch in skeleton.hip
    (``use_tgroup``: threshold mode at depths 2..4 uses the T-group kernel; ``use_screen32``:
    its fp32-screened form k_level_lds_f at the depths of PCG_TG_F32 / PCG_TUNE_SCREEN_MASK)."""
    if d == 0:
        return f"k_level0<{1 if full_p else 0}>"
    if 2 <= d <= 4:   # (full-p mode runs the T-group sweeps too, since round 4)
        mask = 0x18 if screen_mask < 0 else screen_mask
        if (mask >> d) & 1:   # k_level_lds_f<d, WIDE, REC>: REC = the record-routing build
            return f"k_level_lds_f<{d}, false, false>"
        return f"k_level_lds_t<{d}, false>"
    return f"k_level_lds<{d}, {1 if full_p else 0}>"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--samples", type=int, default=10000)
    ap.add_argument("--max-depth", type=int, default=4)
    ap.add_argument("--alpha", type=float, default=0.05)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--full-p", action="store_true", help="compute every p-value (PCG_FLAG_FULL_P)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-full-p", action="store_true", help="skip the full-p comparison run after the timed steps")
    ap.add_argument("--cpu-depth", type=int, default=3, help="depths timed for the CPU port baseline")
    ap.add_argument("--json-extra", action="store_true", help="print per-level detail to stderr")
    ap.add_argument("--workload", choices=["skeleton", "rq2"], default="skeleton",
                    help="skeleton: the headline line (config 5); rq2: every case of an Online-Boutique-shaped "
                         "RQ2 tree through pc_pagerank, cases dealt one per GPU (config 2)")
    ap.add_argument("--rq2-cases", type=int, default=125, help="cases in the synthetic RQ2 tree")
    ap.add_argument("--rq2-prefetch", type=int, default=4,
                    help="loader processes reading / windowing the next cases while the GPU runs the current one")
    ap.add_argument("--rq2-loader", choices=["process", "thread"], default="process")
    ap.add_argument("--rq2-dataset", choices=["online-boutique", "sock-shop"], default="online-boutique",
                    help="shape of the synthetic RQ2 tree (config 2 names both)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="pcg_set_tuning knob for the engine (e.g. NBW=2048; include/pcgpu.h PCG_TUNE_*), A/B runs")
    return ap.parse_args()


def cpu_baseline(X: np.ndarray, alpha: float, depth: int, gpu_tests: list, gpu_removed: np.ndarray,
                 stride: int = 20) -> dict:
    """Oracle C port (pc_oracle.c: LU per test, OpenMP) on this host's cores, on the SAME depth
    mix as the GPU line: depths 0..``depth`` run in full (their removals and per-level test
    counts are checked against the GPU's), each deeper depth timed on a node sample (every
    ``stride``-th node's visits on the graph at the start of that depth — the GPU's, which the
    full-size parity test pins to the oracle's). value = all of the GPU line's unique tests
    over the CPU time projected from the per-depth rates."""
    from oracle import cpc
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    N = X.shape[0]
    C = np.corrcoef(X.T)
    t0 = time.perf_counter()
    ref = cpc.skeleton(C, N, alpha=alpha, max_depth=depth, want_union=False, nthreads=cores)
    full_s = time.perf_counter() - t0
    per_level = []
    est_s = 0.0
    for d, tests in enumerate(gpu_tests):
        if d < ref.levels:
            rate = ref.tests[d] / ref.secs[d]
            per_level.append({"depth": d, "tests": ref.tests[d], "seconds": ref.secs[d], "rate": rate,
                              "how": "full depth"})
        else:
            t_s, sec = cpc.level_sample(C, N, gpu_removed, d, 0, stride, alpha=alpha, nthreads=cores)
            rate = t_s / sec
            per_level.append({"depth": d, "tests": t_s, "seconds": sec, "rate": rate,
                              "how": f"nodes x = 0 mod {stride}"})
        est_s += tests / rate
    total = int(sum(gpu_tests))
    return {"value": total / est_s, "unit": "CI tests/s", "cores": cores, "kind": "port",
            "sample": f"same SEM and depth mix as the GPU line: depths 0..{ref.levels - 1} in full "
                      f"({sum(ref.tests)} unique tests, {full_s:.1f} s), deeper depths on every {stride}-th "
                      f"node's visits; CPU time projected per depth = {est_s:.1f} s for {total} tests",
            "per_level": per_level, "projected_seconds": est_s, "_ref": ref}


def cpu_reference_equiv(X: np.ndarray, ref, budget_s: float = 4.0) -> dict:
    """causal-learn's per-test work (ix_ gather, np.linalg.inv, math.log,
    norm.cdf, dict memo) single-threaded, on a fixed sample of depth-1 tests."""
    from oracle import fisherz
    C = np.corrcoef(X.T)
    N = X.shape[0]
    adj = (ref.removed_level == -1) | (ref.removed_level >= 1)
    np.fill_diagonal(adj, False)
    rng = np.random.default_rng(1)
    xs, ys = np.nonzero(np.triu(adj, 1))
    cache = {}
    count = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        e = int(rng.integers(len(xs)))
        x, y = int(xs[e]), int(ys[e])
        nb = np.nonzero(adj[x])[0]
        s = int(nb[rng.integers(len(nb))])
        if s == y:
            continue
        key = (x, y, (s,))
        if key not in cache:
            cache[key] = fisherz.pvalue(C, N, x, y, (s,))
            count += 1
    dt = time.perf_counter() - t0
    return {"value": count / dt, "cores": 1, "tests": count, "seconds": dt}


OB_PC_PAGERANK_S_PER_CASE = 3.39   # paper Table 6, PC-PageRank, Online Boutique, 8-CPU machine


def rq2_main(args):
    """BASELINE config 2: the RQ2 loop (rcaeval_amd.rq2.run — read_csv, window, preprocess,
    K1 + skeleton + orientation + PageRank, JSON dump) over a synthetic Online-Boutique-shaped
    tree (44 metrics + time per case, 1200 s recorded, windowed to 300 + 300 rows by rq2).
    Cases are dealt round-robin, one process per GPU; value = cases/s of the whole job."""
    import shutil
    import tempfile

    import torch
    from rcaeval_amd import rq2, synth
    from rcaeval_amd.engine import get_engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("gloo")
    get_engine(local)
    base = os.environ.get("PCG_RQ2_DIR") or (tempfile.mkdtemp(prefix="rq2_") if rank == 0 else None)
    if world > 1:      # every rank reads rank 0's tree
        box = [base]
        torch.distributed.broadcast_object_list(box, src=0)
        base = box[0]
    dataset = args.rq2_dataset
    root = os.path.join(base, "data", dataset)
    ss = dataset == "sock-shop"
    services = [s for s in (synth.SS_SERVICES if ss else synth.OB_SERVICES)
                if s not in (("front-end",) if ss else ("frontend", "redis"))]
    faults = ("cpu", "mem", "delay", "loss") if ss else ("cpu", "mem", "delay", "loss", "disk")
    per = max(1, args.rq2_cases // (len(services) * len(faults)))
    if rank == 0 and not os.path.isdir(root):
        synth.write_rq2_dataset(root, services=services, faults=faults, cases=per, rows=1200, seed=args.seed,
                                flavor=dataset)
    if world > 1:
        torch.distributed.barrier()
    out_dir = os.path.join(base, "out")         # one results dir: rank 0 evaluates every rank's cases
    # warm-up on this rank's first case (engine, HIP module load), then the timed pass
    first = rq2.list_cases(root)[rank::world][:1]
    for p in first:
        rq2.process(p, "pc_pagerank", dataset, tempfile.mkdtemp(), length=None)
    from rcaeval_amd import phases
    if args.rq2_loader == "process":
        rq2.start_loaders(args.rq2_prefetch)     # spawned before the timed pass, like the engine itself
    if world > 1:
        torch.distributed.barrier()
    phases.enable()
    t0 = time.perf_counter()
    res = rq2.run(root, "pc_pagerank", dataset, out_dir, rank=rank, world=world, prefetch=args.rq2_prefetch,
                  loader=args.rq2_loader)
    dt = time.perf_counter() - t0
    phases.enable(False)
    rq2.stop_loaders()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    if rank == 0:
        n_cases = res["cases"]
        s_per_case = dt / n_cases
        print(json.dumps({
            "metric": f"PC-PageRank RQ2 cases/s ({dataset}-shaped, cases dealt over GPUs)",
            "value": n_cases / dt, "unit": "cases/s", "n_gpus": world, "steps": 1, "warmup": 1,
            "ms_per_step": 1000.0 * dt, "higher_is_better": True, "scaling": "weak",
            # whole-job cases/s over the published sequential rate (1 / 3.39 s per OB case)
            "vs_baseline": (n_cases / dt) * OB_PC_PAGERANK_S_PER_CASE if not ss else None,
            "dtype": "f64", "data": f"synthetic {dataset}-shaped RQ2 tree (rcaeval_amd.synth.write_rq2_dataset)",
            "config": {"workload": f"rq2.run pc_pagerank over {n_cases} cases ({per} per service x fault), "
                                   "read_csv + window + preprocess + PC + orientation + PageRank + JSON",
                       "parallelism": f"cases round-robin over {world} GPU(s)"},
            "seconds_per_case_per_gpu": s_per_case * world,
            "loaders": f"{args.rq2_prefetch} {args.rq2_loader}es" if args.rq2_prefetch else "none (sequential)",
            # rank 0's cases: wall ms per case of each phase (read_csv / window run on the loader
            # threads when prefetch > 0, overlapped with the GPU work of the previous case)
            "phase_ms_per_case": {k: round(1000.0 * v[0] / max(res["my_cases"], 1), 4)
                                  for k, v in sorted(res.get("phases", {}).items(), key=lambda kv: -kv[1][0])},
            "published_seconds_per_case_cpu": OB_PC_PAGERANK_S_PER_CASE,
            "summary": res["summary"]}), flush=True)
    if not os.environ.get("PCG_RQ2_DIR") and rank == 0:
        shutil.rmtree(base, ignore_errors=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    args = parse()
    if args.workload == "rq2":
        return rq2_main(args)
    import torch
    from rcaeval_amd import _lib, synth
    from rcaeval_amd.engine import get_engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (default off): several ranks on one GPU need gloo + a shared device
    device = int(os.environ.get("PCG_BENCH_DEVICE", local))
    backend = os.environ.get("PCG_DIST_BACKEND", "nccl")
    # PCG_BENCH_FORCE_DIST=1: run the sharded driver even at world 1 (its overhead, measured)
    dist_path = world > 1 or os.environ.get("PCG_BENCH_FORCE_DIST") == "1"
    if dist_path:
        import torch.distributed as dist
        torch.cuda.set_device(device)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)
    eng = get_engine(device)
    for kv in args.tune:
        k, v = kv.split("=", 1)
        eng.set_tuning(k, int(v, 0))
    flags = _lib.PCG_FLAG_FULL_P if args.full_p else 0

    X = synth.gaussian_sem(args.n, args.samples, seed=args.seed)
    Xd = eng.to_device(X)                      # resident in HBM before timing
    torch.cuda.synchronize()

    phases = []

    # default for N > 1: the level loop and its collectives run in C (pcg_skeleton_sharded on an
    # RCCL communicator of the library's own: one host round trip per depth, no Python in the
    # loop; at world 1 it adds 0.56 ms per step to the single-GPU call where the torch.distributed
    # driver adds 1.58 ms). PCG_DIST_NATIVE=0 selects the torch.distributed driver; so does a
    # communicator that fails to come up on any rank (agreed collectively, no rank left waiting).
    native = dist_path and os.environ.get("PCG_DIST_NATIVE", "1") == "1"
    if native:
        from rcaeval_amd.dist import native_comm
        ok = 1
        try:
            native_comm(eng)
        except Exception as e:   # noqa: BLE001 - fall back to the torch.distributed driver
            print(f"[rank {rank}] native RCCL driver unavailable ({e}); using torch.distributed", file=sys.stderr)
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int32, device=eng.device if backend == "nccl" else "cpu")
        torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MIN)
        native = bool(flag.item())

    k1_events = []

    def one_step():
        t0 = time.perf_counter()
        if native:
            # stream-ordered, no host sync between K1 and the skeleton; K1's time from events on
            # the handle's stream, read after the step
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(eng.stream)
            C = eng.corr_sharded(Xd)
            ev[1].record(eng.stream)
            k1_events.append(ev)
            return eng.skeleton_sharded(C, args.samples, alpha=args.alpha, max_depth=args.max_depth, flags=flags)
        elif dist_path:
            from rcaeval_amd.dist import sharded_corr
            C = sharded_corr(eng, Xd)
        else:   # single GPU: K1 + skeleton in one C call (pcg_pc_skeleton), no host round trip between
            return eng.corr_skeleton(Xd, alpha=args.alpha, max_depth=args.max_depth, flags=flags)[0]
        torch.cuda.synchronize()
        phases.append(("corr", time.perf_counter() - t0))
        if dist_path:
            from rcaeval_amd.dist import sharded_skeleton
            trace = [] if os.environ.get("PCG_DIST_TRACE") else None
            out = sharded_skeleton(eng, C, args.samples, alpha=args.alpha, max_depth=args.max_depth,
                                   flags=flags, trace=trace)
            if trace is not None:
                print(f"[rank {rank}] " + " ".join(f"{p}{d if d >= 0 else ''}={1000 * t:.2f}"
                                                    for p, d, t in trace), file=sys.stderr, flush=True)
            return out
        return eng.skeleton(C, args.samples, alpha=args.alpha, max_depth=args.max_depth, flags=flags)

    def barrier():
        torch.cuda.synchronize()
        if dist_path:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    def progress(msg):
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    for w in range(args.warmup):
        t0 = time.perf_counter()
        one_step()
        torch.cuda.synchronize()
        progress(f"warmup {w}: {1000 * (time.perf_counter() - t0):.2f} ms")
    times, out = [], None
    for _ in range(args.steps):
        out = None          # the previous step's result is released, as a caller consuming each result would
        barrier()
        t0 = time.perf_counter()
        out = one_step()
        barrier()
        dt = time.perf_counter() - t0
        if os.environ.get("PCG_DIST_TRACE"):
            print(f"[rank {rank}] step {1000 * dt:.2f} ms", file=sys.stderr, flush=True)
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=eng.device)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            dt = float(t.item())
        times.append(dt)
        progress(f"step {len(times) - 1}: {1000 * dt:.3f} ms")
    st = out.stats
    tests_total = int(sum(st["tests"]))
    ms = 1000.0 * float(np.mean(times))
    value = tests_total / (ms / 1000.0)

    # dominant kernel: the CI-test kernel of the deepest, largest level
    dmax = int(np.argmax(st["tests"]))
    k_ms = st["kernel_ms"][dmax]
    kname = dominant_kernel(dmax, args.full_p, eng.get_tuning("SCREEN_MASK"))
    roof = roofline_of(kname, int(st["tests"][dmax]), dmax, k_ms)
    if world == 1:      # K1 alone (for its roofline), outside the timed steps
        for _ in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.corr(Xd)
            torch.cuda.synchronize()
            phases.append(("corr", time.perf_counter() - t0))
        corr_med = float(np.median([1000 * t for n_, t in phases if n_ == "corr"][1:]))
    elif native:
        torch.cuda.synchronize()
        for e0, e1 in k1_events:
            phases.append(("corr", e0.elapsed_time(e1) / 1000.0))
        corr_med = float(np.median([1000 * t for n_, t in phases if n_ == "corr"][args.warmup:] or [0.0]))
    else:
        corr_med = float(np.median([1000 * t for n_, t in phases if n_ == "corr"][args.warmup:] or [0.0]))
    k1_tune = {k: eng.get_tuning(k) for k in ("K1_I8", "K1_CRT", "K1_CRT_MINN", "K1_CRT_BITS")}
    roof["k1"] = k1_roofline(args.n, args.samples, corr_med, k1_tune) if corr_med > 0 else None

    # the p-value mode (PCG_FLAG_FULL_P | PCG_FLAG_RECORD) after the timed steps: the same skeleton
    # with the reference-arithmetic p of every test of a 1-in-4099 pair SAMPLE recorded (the
    # parity test's sample; the exact path computes those p with numpy.linalg.inv's LU), the
    # threshold decisions elsewhere — NOT every test's p (pcgpu.h PCG_FLAG_FULL_P). Twice: the
    # first call sizes the exact-path list
    full_p = None
    if not args.full_p and not args.no_full_p and world == 1:
        progress("full-p comparison run")
        C = eng.corr(Xd)
        fl = _lib.PCG_FLAG_FULL_P | _lib.PCG_FLAG_RECORD
        for _ in range(2):
            o = eng.skeleton(C, args.samples, alpha=args.alpha, max_depth=args.max_depth, flags=fl,
                             record_capacity=4_000_000, record_sample=(4099, 17))
        fp_ms = float(sum(o.stats["level_ms"]))
        same = bool(np.array_equal(o.removed_level, out.removed_level)) and o.stats["tests"] == st["tests"]
        full_p = {"what": "sampled records: the reference p of every test of a 1-in-4099 pair sample, "
                          "threshold decisions elsewhere (not every test's p)",
                  "skeleton_device_ms": fp_ms, "tests_per_s": sum(o.stats["tests"]) / (fp_ms / 1e3),
                  "flags": "FULL_P|RECORD, record_sample=(4099, 17)", "records": int(len(o.records)),
                  "kernel_ms_per_level": [round(v, 3) for v in o.stats["kernel_ms"]],
                  "level_ms": [round(v, 3) for v in o.stats["level_ms"]],
                  "exact_path": o.stats["exact"], "same_skeleton_as_threshold": same}

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "CI tests/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic Gaussian SEM (rcaeval_amd.synth.gaussian_sem), resident in HBM",
            "config": {"workload": f"stable PC-fisherz skeleton, {args.n} vars x {args.samples} samples, "
                                   f"max depth {args.max_depth}, alpha {args.alpha}, seed {args.seed}, "
                                   f"ER DAG p=2/(n-1), weights +-U(0.1,0.5)",
                       "parallelism": (f"edge-sharded x{world}" + (" (native RCCL driver)" if native else ""))
                                      if world > 1 else "single GPU",
                       "decision": "full p-value" if args.full_p else "threshold + exact band",
                       **({"tuning": args.tune} if args.tune else {})},
            "skeleton_ms": ms,
            "step_ms_all": [round(1000 * t, 3) for t in times],
            "corr_ms": [round(1000 * t, 3) for n_, t in phases if n_ == "corr"],
            "engine_phases_ms": getattr(out, "extra", {}),
            "tests_per_level": st["tests"], "calls_per_level": st["calls"],
            "kernel_ms_per_level": [round(v, 3) for v in st["kernel_ms"]],
            "level_ms": [round(v, 3) for v in st["level_ms"]],
            "edges_after": st["edges_after"], "exact_path": st["exact"], "screened": st["screened"], "near_alpha": st["near_alpha"], "indep_per_level": st["indep"],
            "roofline": roof,
            "sampled_records": full_p,
        }
        if not args.no_cpu_baseline and world == 1:
            progress("CPU baseline")
            cb = cpu_baseline(X, args.alpha, args.cpu_depth, st["tests"], out.removed_level)
            ref = cb.pop("_ref")
            # parity of the timed GPU run on the CPU-sampled depths
            Lc = ref.levels
            same = bool(np.array_equal(
                np.where(ref.removed_level >= 0, ref.removed_level, -1),
                np.where((out.removed_level >= 0) & (out.removed_level < Lc), out.removed_level, -1)))
            cb["parity_depths_0_%d" % (Lc - 1)] = same and st["tests"][:Lc] == ref.tests
            ce = cpu_reference_equiv(X, ref)
            cb["reference_equivalent_1core_tests_per_s"] = ce["value"]
            line["cpu_baseline"] = cb
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
