#!/usr/bin/env python3
"""bench.py -- all-pairs AJI matrix fill on MI355X (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W
    (N > 1: one rank per GPU -- under torch.distributed.run, or, started
    plainly, bench.py spawns its own N rank processes before any GPU call)

Workload (BASELINE.json metric "10k-genome all-vs-all"): a synthetic
10,000-genome x 100-SCP database (SURVEY.md §8d SYN generator, seed
20250213), all-vs-all AJI.  Every rank generates the same DB (deterministic),
loads it into HBM once (pfaai_load), and owns a contiguous block of output
rows balanced by a measured row-cost model (parfastaai_amd/shard.py).  One
step = the hot path over the resident inputs: the run-table build k_blk (the
reference's E construction, without E) + the scatter/Jaccard/AJI row kernel
k_rows_pl over the rank's rows; for N > 1 the rank's fp64 AJI block is
gathered to rank 0 over RCCL asynchronously, double-buffered so that step
i + 1 computes while step i's gather is in flight (every step computes and
gathers its whole block; the timed region ends after the last gather), and
--chunks > 1 also cuts a step's rows into pipeline chunks, each gathered as
soon as it is computed (the run table built once per step).
Total work is fixed as N grows: scaling "strong".  value = genome pairs of
the whole matrix / max step time over ranks.

Extra JSON objects:
  roofline      dominant kernel k_rows_pl: algorithmic bytes per launch
                (8 B per E event + 8 B per AJI written) / its mean
                duration from HIP events on the launch stream over the timed
                region; peak 8 TB/s HBM; traffic from the committed rocprofv3
                PMC summary (profiles/) when present.
  cpu_baseline  the reference CLI (oracle/_ref/par_fastaai.x, built from its
                own sources) on a bounded SYN sample, rank 0 at N = 1 only;
                falls back to the CPU oracle ("port") if the binary is absent.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

E2E_PROFILE = "r06/final/e2e_c2.json"  # tools/gpu/e2e_c2.py's latest committed run (README quotes the same file)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "genome-pairs/sec (AJI matrix fill) + achieved HBM GB/s, 10k-genome all-vs-all"
ROWS_KERNEL = ("pfaai::k_rows_pl (fused scatter + Jaccard + AJI; the wide rows as 1024-thread workgroups, the "
               "rows of <= 2047 columns as 512-thread ones on a second stream, one pfaai_run)")


def log(msg):
    print(f"[bench r{os.environ.get('RANK', '0')}] {msg}", file=sys.stderr, flush=True)


def pmc_profile(genomes, prot, world):
    """profiles/pmc_k_rows.json (tools/pmc_summary.py from rocprofv3 --pmc
    passes over one k_rows_pl launch on all rows of the 10k x 100 workload):
    HBM bytes per launch (FETCH_SIZE + WRITE_SIZE), VALU-busy fraction, wave
    wait fraction, LDS bank-conflict fraction.  Other shapes: None."""
    p = os.path.join(ROOT, "profiles", "pmc_k_rows.json")
    if not os.path.exists(p) or (genomes, prot, world) != (10000, 100, 1):
        return None
    try:
        with open(p) as f:
            return json.load(f)
    except Exception:
        return None


def traffic_from_profiles(genomes, prot, world):
    """HBM bytes per k_rows_pl launch (pmc_profile), or None."""
    d = pmc_profile(genomes, prot, world)
    return d.get("hbm_bytes_per_launch") if d else None


def cgroup_cpus():
    """CPUs of this process's cgroup CPU quota (cgroup v2 cpu.max / v1
    cfs_quota), None if unlimited or unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else round(q / per, 2)
    except (OSError, ValueError):
        return None


def usable_cpus():
    """CPUs this process can actually run on: its affinity set, capped by its
    cgroup CPU quota.  (On the GPU box the affinity lists 256 CPUs but the
    quota is 16: the reference at 256 OpenMP threads ran C2 in 131.5 s vs
    112.8 s at 16 -- oversubscribed, its parallel loader phases slowed 3-7x,
    profiles/r03a_e2e_c2_threads256.json -- so 256 would understate it.)"""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q = cgroup_cpus()
    return max(1, min(n, int(q))) if q else n


def host_info(threads):
    """The CPU the baseline ran on: model name, logical CPUs of the machine,
    CPUs this process may run on (affinity), the cgroup's CPU quota (the
    box's share can be far smaller than both), threads the baseline was
    given."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": affinity, "usable_cpus": usable_cpus(),
            "cgroup_cpu_quota": cgroup_cpus(), "threads_used": threads}


def c2_reference():
    """The end-to-end C2 comparison (2,000 genomes, SQLite DB -> CSV) of our
    CLI, the reference-side drop-in and the reference, medians of repeated
    runs by tools/gpu/e2e_c2.py, committed under profiles/."""
    p = os.path.join(ROOT, "profiles", E2E_PROFILE)
    try:
        with open(p) as f:
            d = json.load(f)
        return {"source": "profiles/" + E2E_PROFILE, "genomes": d["genomes"], "repeats": d.get("repeats", 1),
                "reference_wall_s": d["reference_wall_s"], "reference_threads": d["reference_threads"],
                "ours_wall_s": d["ours_wall_s"], "dropin_wall_s": d.get("dropin_wall_s"),
                "csv_byte_identical": d["csv_byte_identical"]}
    except (OSError, KeyError, ValueError):
        return None


def run_reference(ref, db, threads, timeout=900):
    """The reference CLI on one SQLite DB; its own phase timers (interface.hpp:
    309-325, algorithm_impl.hpp:304).  A heartbeat line every 30 s."""
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    t0 = time.perf_counter()
    with tempfile.TemporaryDirectory() as td:
        p = subprocess.Popen([ref, db, os.path.join(td, "out.csv")], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                             text=True, env=env)
        while True:
            try:
                out, _ = p.communicate(timeout=30)
                break
            except subprocess.TimeoutExpired:
                if time.perf_counter() - t0 > timeout:
                    p.kill()
                    raise RuntimeError("reference timed out")
                log(f"cpu baseline: reference running {time.perf_counter() - t0:.0f}s")
    wall = time.perf_counter() - t0
    if p.returncode != 0:
        raise RuntimeError(f"reference exited {p.returncode}")

    def ms(label):
        m = re.search(re.escape(label) + r"\s*:\s*([0-9.e+]+) ms", out)
        return float(m.group(1)) if m else None

    e_ms, jac_ms = ms("E constr.   (fin)"), ms("JAC Construction")
    return {"hot_s": (e_ms + jac_ms) / 1e3, "e_constr_s": e_ms / 1e3, "jac_s": jac_ms / 1e3, "wall_s": wall}


def cpu_baseline(n_prot=100, c2_genomes=2000, sample_genomes=320, quick=False):
    """The reference CLI (built from its own sources) timed on this host's
    cores with OMP_NUM_THREADS = the CPUs this process can use (affinity
    capped by the cgroup quota; BASELINE.md plan): at config C2 (SYN 2,000 x 100 -- the largest config the reference
    can run) unless quick, and on the N = 320 sample (secondary field).
    Hot path = its own 'E constr. (fin)' + 'JAC Construction' timers.  Falls
    back to the CPU oracle ("port") where the binary is absent."""
    from parfastaai_amd import syn

    ref = os.path.join(ROOT, "oracle", "_ref", "par_fastaai.x")
    threads = usable_cpus()
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from parfastaai_amd.datastruct import ParFAAIData

    def sizes(n):  # |F| and the reference's |E| (countTetramerTuples, ds_helper.hpp:206-265) of SYN n x P
        g = syn.generate(n, n_prot)
        ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"])
        return len(g["F_genome"]), O.Problem(ds.problem()).count_e(), ds

    if os.path.exists(ref):
        def measure(n):
            n_f, n_e, _ = sizes(n)
            pairs = n * (n - 1) // 2
            with tempfile.TemporaryDirectory() as td:
                db = os.path.join(td, "syn.db")
                t0 = time.perf_counter()
                syn.write_db(db, n, n_prot)
                log(f"cpu baseline: SYN {n} x {n_prot} DB written in {time.perf_counter() - t0:.1f}s")
                r = run_reference(ref, db, threads)
            b_alg = 8 * n_e + 4 * n_f + 8 * pairs
            return {"genomes": n, "pairs": pairs, "events": n_e, "F": n_f, "hot_s": round(r["hot_s"], 3),
                    "e_constr_s": round(r["e_constr_s"], 3), "jac_s": round(r["jac_s"], 3),
                    "wall_s": round(r["wall_s"], 2), "pairs_per_s": round(pairs / r["hot_s"], 1),
                    "events_per_s": round(n_e / r["hot_s"], 1), "alg_GBps": round(b_alg / r["hot_s"] / 1e9, 3)}

        small = measure(sample_genomes)
        main = small if quick else measure(c2_genomes)
        return {"value": main["pairs_per_s"], "unit": "genome-pairs/s", "cores": threads, "kind": "reference",
                "sample": f"reference par_fastaai.x (built from its own sources) on SYN N={main['genomes']} "
                          f"P={n_prot} all-vs-all ({'config C2' if not quick else 'quick sample'}), "
                          f"OMP_NUM_THREADS={threads} (this process's usable CPUs: affinity capped by the cgroup quota); hot path = its own "
                          f"'E constr. (fin)' + 'JAC Construction' timers = {main['hot_s']:.2f} s "
                          f"(wall incl. SQLite + CSV {main['wall_s']:.1f} s)",
                "c2": None if quick else main, "secondary_sample": small, "host": host_info(threads),
                "c2_end_to_end": c2_reference()}
    # fallback: the CPU oracle (single thread restatement of the reference)
    n_f, n_e, ds = sizes(sample_genomes)
    pairs = sample_genomes * (sample_genomes - 1) // 2
    t0 = time.perf_counter()
    O.Problem(ds.problem()).ref_run()
    dt = time.perf_counter() - t0
    return {"value": pairs / dt, "unit": "genome-pairs/s", "cores": 1, "kind": "port",
            "sample": f"CPU oracle (E build + radix sort + extents + JAC) on SYN N={sample_genomes} P={n_prot}, "
                      f"{dt:.2f} s", "host": host_info(1), "c2_end_to_end": c2_reference()}


def free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv):
    """`python bench.py --gpus N` (N > 1) started without a launcher: start N
    child processes of this script, rank r on GPU r (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their environment),
    and return the worst exit code.  The parent never touches the GPU (it has
    not even imported torch) and replaces no process: the children are
    ordinary subprocesses.  If one rank fails, the others are stopped."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PFAAI_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for r, p in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):  # a rank died: the others would wait at a collective forever
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    p.terminate()
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    try:
                        rcs[r] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[r] = p.wait()
            break
        time.sleep(0.05)
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        log(f"rank exit codes {rcs}")
    return bad[0] if bad else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--genomes", type=int, default=10000)
    ap.add_argument("--prot", type=int, default=100)
    ap.add_argument("--cpu-baseline", choices=["auto", "quick", "none"], default="auto",
                    help="auto: the reference at config C2 (~2 min) + the N=320 sample; quick: the sample only")
    ap.add_argument("--cpu-sample", type=int, default=320)
    ap.add_argument("--chunks", type=int, default=1,
                    help="pipeline chunks per rank and step (gather of chunk j overlaps chunk j+1); "
                         "default 1: the gather overlaps the next step instead (tools/gpu/shard_times.py: "
                         "2 chunks add 0.38 ms of launch tails per 10k/8 shard, 4 chunks 0.87 ms)")
    ap.add_argument("--slots", type=int, default=None,
                    help="AJI buffer sets per rank: 2 (default at N > 1) lets step i + 1 compute while "
                         "step i's gather is in flight; 1 waits for each step's gather")
    ap.add_argument("--rehearse-gloo", action="store_true",
                    help="one-GPU box rehearsal of the N > 1 flow (split, spans, pipelined gather, reassembly, "
                         "result check): gloo instead of RCCL, every rank on device local %% device_count, the "
                         "gather through host buffers -- not a measurement")
    ap.add_argument("--split", choices=["cyclic", "contiguous"], default="contiguous",
                    help="N > 1: rank r runs one contiguous cost-balanced row block (contiguous, the default), or "
                         "in ONE launch over its row list (pfaai_set_row_order) the 32-row groups dealt to it in "
                         "snake order (cyclic: every rank gets the whole matrix's mix of wide and narrow rows; its "
                         "rows' JAC segments go straight into rank 0's output by grouped send / recv).  The one-GPU "
                         "emulation (profiles/r06/shard_cyclic.txt) put the slowest cyclic rank at 1.08 ms against "
                         "1.05-1.09 contiguous, so the default stays contiguous")
    ap.add_argument("--rccl-one-gpu", action="store_true",
                    help="one-GPU box rehearsal of the N > 1 flow through RCCL itself (the nccl backend): every rank "
                         "on device local %% device_count with its own NCCL_HOSTID, so RCCL takes the ranks for "
                         "separate hosts (it refuses two ranks of one host on one device) and moves the data over "
                         "its socket transport on the loopback interface instead of xGMI -- the RCCL send / recv / "
                         "gather paths execute; not a measurement")
    ap.add_argument("--f-only", action="store_true",
                    help="give the engine F only (device radix-sort transposition instead of G)")
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="launcher check without a GPU: every rank prints its RANK / WORLD_SIZE / LOCAL_RANK "
                         "as one JSON line and exits before any GPU call")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: spawn the N ranks here, before anything touches the GPU
        return spawn_ranks(args.gpus, sys.argv[1:])
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:  # never measure a different number of GPUs than asked for
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={world}")
        return 2
    if args.launch_dry_run:
        print(json.dumps({"rank": rank, "world_size": world, "local_rank": local,
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}), flush=True)
        return 0
    import torch  # (first: one HIP runtime per process)
    import torch.distributed as dist

    rehearse = args.rehearse_gloo and world > 1
    one_gpu = args.rccl_one_gpu and world > 1 and not rehearse
    if rehearse or one_gpu:  # (RCCL refuses two ranks of one host on one device; gloo gathers host tensors)
        local = local % max(1, torch.cuda.device_count())
    if one_gpu:  # read by RCCL at its first communicator: one "host" per rank, loopback sockets
        os.environ["NCCL_HOSTID"] = f"pfaai-bench-rank{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    hdev = torch.device("cpu") if rehearse else dev  # where the gathered blocks and reductions live
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        if rank == 0:
            ver = ".".join(map(str, torch.cuda.nccl.version())) if not rehearse else "-"
            log(f"communicator: backend {dist.get_backend()} (RCCL {ver}), size {dist.get_world_size()}")

    from parfastaai_amd import _capi, syn
    from parfastaai_amd.datastruct import ParFAAIData
    from parfastaai_amd.shard import PipelinedGather, SegmentGather, cyclic_rows, jac_segments, split_range, split_rows

    t0 = time.perf_counter()
    g = syn.generate(args.genomes, args.prot)
    n_f = len(g["F_genome"])
    log(f"generated SYN N={args.genomes} P={args.prot} |F|={n_f} in {time.perf_counter() - t0:.1f}s")
    ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"])
    if not args.f_only:  # the DB's genome-major <p>_genomes lists: the row kernel walks them
        ds.with_genome_major(g["G_off"], g["G_tet"])
    eng = _capi.Engine(local)
    # a rank loads the whole input but builds the walk data (G_pos / G_end,
    # the run-end sort) of its own row block only (pfaai_load_rows); all-vs-all
    # rows are genomes, so the blocks are known before the load
    # (cus: cuts a few rows past a round of 2 x CUs row workgroups move back)
    blocks = split_rows(args.genomes, world, cus=torch.cuda.get_device_properties(dev).multi_processor_count)
    # block-cyclic (--split cyclic): the rank's rows are spread over the
    # whole matrix, so it loads every genome's walk data (pfaai_load)
    cyclic = world > 1 and args.split == "cyclic" and not args.f_only
    lists = cyclic_rows(args.genomes, world) if cyclic else None
    t0 = time.perf_counter()
    eng.load(**ds.problem(), rows=blocks[rank] if world > 1 and not cyclic else None)
    load_wall_ms = (time.perf_counter() - t0) * 1e3
    del g
    ms_checks, ms_upload, ms_load_dev = eng.load_timing()
    load_path = eng.load_info()
    log(f"pfaai_load {load_wall_ms:.0f} ms (host checks {ms_checks:.0f}, H2D {ms_upload:.0f}, device {load_path} "
        f"{ms_load_dev:.2f} ms)")
    n_rows, n_pairs = eng.shape()
    assert n_rows == args.genomes
    if cyclic:
        segs = [jac_segments(args.genomes, rl) for rl in lists]
        eng.set_row_order(lists[rank])
        count = sum(l - f for f, l in segs[rank])  # the rank's pairs
    else:
        spans = [eng.row_span(rb, re) for rb, re in blocks]
        first, count = spans[rank]
    # N > 1: the rank's AJI block is gathered to rank 0 (RCCL, async); with
    # two buffer sets the gather of step i overlaps the compute of step i + 1.
    # --chunks > 1: the rows in pipeline chunks, chunk j gathered while chunk
    # j + 1 computes; the run table is built by chunk 0 only (PFAAI_FLAG_KEEP_RUNS)
    nch = max(1, args.chunks)
    slots = max(1, args.slots) if args.slots else (1 if world == 1 else 2)
    stream = torch.cuda.current_stream(dev)
    n_steps = [0]
    if cyclic:
        if nch != 1:
            raise SystemExit("--chunks applies to --split contiguous")
        # every rank runs its list into a full-size JAC-ordered array; rank
        # 0's is the output (rehearsal: a device twin of each host array)
        pg = SegmentGather(segs, n_pairs, dst=0, device=hdev, slots=slots)
        dfull = [torch.zeros_like(b, device=dev) for b in pg.slot_bufs] if rehearse else pg.slot_bufs
        my_rows = len(lists[rank])
        sub = [[(0, my_rows)]]  # (the |E| pass below: one launch over the list)
        bases = [[dfull[k].data_ptr()] for k in range(slots)]
    else:
        sub = [split_range(b0, b1, nch, n_rows) for b0, b1 in blocks]
        counts = [[eng.row_span(c0, c1)[1] for c0, c1 in s] for s in sub]
        pg = PipelinedGather(counts, dst=0, device=hdev, slots=slots)
        # pfaai_run indexes by the global JAC index: chunk j writes its own buffer
        # (rehearsal: a device twin of each host gather buffer)
        dbufs = [[torch.zeros_like(b, device=dev) for b in bs] for bs in pg.slot_bufs] if rehearse else pg.slot_bufs
        bases = [[dbufs[k][j].data_ptr() - eng.row_span(c0, c1)[0] * 8 for j, (c0, c1) in enumerate(sub[rank])]
                 for k in range(slots)]

    def step_cyclic():
        i = n_steps[0]
        n_steps[0] += 1
        pg.begin(i)  # buffer set i % slots: the stream waits for the transfers that last read it
        eng.run(0, my_rows, 0, bases[i % slots][0], stream=stream.cuda_stream)
        if rehearse:
            pg.buf.copy_(dfull[i % slots])
        pg.issue()
        if slots == 1:
            pg.wait()

    def step():
        if cyclic:
            return step_cyclic()
        i = n_steps[0]
        n_steps[0] += 1
        pg.begin(i)  # buffer set i % slots: the stream waits for the gathers that last read it
        for j, (c0, c1) in enumerate(sub[rank]):
            if c1 > c0:
                eng.run(c0, c1, _capi.FLAG_KEEP_RUNS if j else 0, bases[i % slots][j], stream=stream.cuda_stream)
            if rehearse:
                pg.bufs[j].copy_(dbufs[i % slots][j])
            pg.issue(j)
        if slots == 1:
            pg.wait()

    def barrier():
        if world > 1:
            if rehearse:
                dist.barrier()
            else:
                dist.barrier(device_ids=[local])

    # |E| of this rank's rows: one untimed pass, chunk by chunk -- also the
    # one-shot cost: the load's device build + this first step
    eng.timing(reset=True)
    n_events = 0
    for j, (c0, c1) in enumerate(sub[0] if cyclic else sub[rank]):
        if c1 > c0:
            eng.run(c0, c1, 0, bases[0][j], stream=stream.cuda_stream)
            torch.cuda.synchronize(dev)
            n_events += eng.stats()["n_events"]
    first_wall_ms = (time.perf_counter() - t0) * 1e3  # since the load began
    _, fb, fr = eng.timing(reset=True)
    first_step_ms = fb + fr
    for _ in range(args.warmup):
        step()
    pg.wait()
    torch.cuda.synchronize(dev)
    barrier()
    eng.timing(reset=True)

    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    pg.wait()  # every step's gather has landed on rank 0
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    n_runs, ms_build, ms_rows = eng.timing(reset=True)
    # per step: the rank's k_blk (once) and its k_rows_pl launches (one per chunk)
    n_runs = args.steps
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=hdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        ev = torch.tensor([n_events], dtype=torch.int64, device=hdev)
        dist.all_reduce(ev)
        total_events = int(ev.item())
        km = torch.tensor([ms_rows / max(n_runs, 1), ms_build / max(n_runs, 1), ms_load_dev + first_step_ms,
                           ms_load_dev], dtype=torch.float64, device=hdev)
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        k_rows_ms_max, k_build_ms_max, one_shot_ms, load_ms_max = km.tolist()
    else:
        total_events = n_events
        one_shot_ms = ms_load_dev + first_step_ms
        load_ms_max = ms_load_dev
        k_rows_ms_max = ms_rows / max(n_runs, 1)
        k_build_ms_max = ms_build / max(n_runs, 1)
    ms_per_step = elapsed * 1e3 / args.steps

    if rank == 0:
        # spot-check the gathered / local result for sanity (cheap properties)
        vals = pg.result()
        vmin, vmax = float(vals.min().item()), float(vals.max().item())
        assert vals.numel() == n_pairs and 0.0 <= vmin and vmax <= 1.0, (vals.numel(), vmin, vmax)
        if world > 1:  # the gathered row blocks equal one run over all rows on this device, bit for bit
            eng.load(**ds.problem())  # (the whole input's walk data: this rank loaded its block only)
            full = torch.empty(n_pairs, dtype=torch.float64, device=dev)
            eng.run(0, n_rows, 0, full.data_ptr(), stream=stream.cuda_stream)
            torch.cuda.synchronize(dev)
            assert torch.equal(full.to(vals.device), vals), "gathered AJI differs from a single-device run"
            # the other buffer set of the double-buffered gather (the step before the last)
            checked = [pg.cur]
            if slots > 1 and args.steps + args.warmup >= 2:
                k = (n_steps[0] - 2) % slots
                assert torch.equal(full.to(vals.device), pg.result(slot=k)), f"gathered AJI of buffer set {k} differs"
                checked.append(k)
            del full
            log(f"gathered AJI (buffer sets {checked}) equals a single-device run over all rows (bit-exact)")

        k_rows_ms = ms_rows / max(n_runs, 1)  # rank 0's own k_rows launch(es) per step
        rank_pairs = count
        alg_bytes = 8 * n_events + 8 * rank_pairs
        achieved = alg_bytes / (k_rows_ms * 1e-3) / 1e9
        step_bytes = 8 * total_events + 4 * n_f + 8 * n_pairs  # SURVEY §8d B_alg
        # priced against HBM (the contract's roofline); what actually limits the
        # kernel comes from the committed counters: the HBM traffic it causes
        # is a fraction of its algorithmic bytes (member lines shared through
        # L2), while its SIMDs issue VALU most of the time (S5's fp64
        # divisions, the member scatter) and its waves wait on the per-protein
        # load chain and barrier -- "valu+latency" 
        pmc = pmc_profile(args.genomes, args.prot, world) or {}
        traffic = pmc.get("hbm_bytes_per_launch")
        valu_busy = pmc.get("valu_busy")
        bound = "hbm"
        if traffic and valu_busy and traffic < 0.5 * alg_bytes and valu_busy > 0.5:
            bound = "valu+latency"
        roofline = {"bound": bound, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "peak_basis": "hbm 8 TB/s (algorithmic bytes / kernel time)",
                    "traffic_over_alg": round(traffic / alg_bytes, 3) if traffic else None,
                    "valu_busy": round(valu_busy, 3) if valu_busy else None,
                    "wave_frac_waiting": pmc.get("wave_frac_waiting"),
                    "valu_insts": pmc.get("valu_insts"), "salu_insts": pmc.get("salu_insts"),
                    "pmc_source": ("profiles/pmc_k_rows.json (" + str(pmc.get("tag")) + ")") if pmc else None,
                    "kernel": ROWS_KERNEL,
                    "kernel_ms": round(k_rows_ms, 4), "alg_bytes_per_launch": alg_bytes,
                    "build_kernels_ms": round(ms_build / max(n_runs, 1), 4)}
        # the one-shot load: the device F / G transposition and the per-entry
        # run ends (SURVEY §8d timed region starts after it; reported here,
        # never in `value`).  Algorithmic bytes per F entry of the both-given
        # check (G_CHECKED): read its (protein, genome) 8 B + the caller's G_tet
        # 4 B, write G_pos 4 B, G_end 4 B and the u16 protein column 2 B = 22 B;
        # the two-pass sort moves ~50 B (pfaai_sort.hpp: per pass a histogram
        # read + a read and a write of 8-B records)
        alg_per_f = {"g_checked": 22, "g_from_f": 26, "f_from_g": 22}.get(load_path)
        # the bytes the implemented passes move per F entry (G_CHECKED, the
        # run-end sort): hist 1 reads F 8 + writes the u16 column 2; scatter 1
        # reads F 8, writes a record 8; hist 2 reads 8; scatter 2 reads 8,
        # writes G_pos 4 + G_end 4; beside them k_hash_f reads F 8 and the G
        # side of the check G_tet 4 = 62 B
        pass_per_f = {"g_checked": 62}.get(load_path) if world == 1 else None
        load = {"path": load_path, "device_ms": round(ms_load_dev, 3), "host_checks_ms": round(ms_checks, 1),
                "h2d_ms": round(ms_upload, 1), "wall_ms": round(load_wall_ms, 1), "F": n_f,
                "alg_bytes_per_F": alg_per_f,
                "alg_GBps": round(alg_per_f * n_f / (ms_load_dev * 1e-3) / 1e9, 1) if alg_per_f else None,
                "frac": round(alg_per_f * n_f / (ms_load_dev * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if alg_per_f else None,
                "pass_bytes_per_F": pass_per_f,
                "pass_frac": round(pass_per_f * n_f / (ms_load_dev * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if pass_per_f else None,
                "device_ms_max_rank": round(load_ms_max, 3),
                "rows": ("all (block-cyclic ranks)" if cyclic else
                         f"rank 0 of {world}: walk data of rows {list(blocks[rank])}") if world > 1 else "all",
                "one_shot_ms": round(ms_load_dev + first_step_ms, 3), "first_step_ms": round(first_step_ms, 3),
                "one_shot_wall_ms": round(first_wall_ms, 1)}
        cpu = None
        if args.cpu_baseline != "none" and world == 1:
            try:
                log("cpu baseline ...")
                cpu = cpu_baseline(args.prot, sample_genomes=args.cpu_sample, quick=args.cpu_baseline == "quick")
            except Exception as e:  # reported, never fatal
                cpu = {"value": None, "error": str(e)}
        line = {
            "metric": METRIC,
            "value": round(n_pairs / (ms_per_step * 1e-3), 1),
            "unit": "genome-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            # one fill from the raw input arrays already in HBM: the load's
            # device build (F / G transposition, G_pos, G_end, the both-given
            # check) + the first step (SURVEY §8d's timed region starts after
            # the load; this puts the load's cost beside `value`)
            "value_one_shot": round(n_pairs / (one_shot_ms * 1e-3), 1),
            "one_shot_ms": round(one_shot_ms, 4),  # (max over ranks)
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "i32+f64",
            "data": "synthetic",
            "config": {"workload": f"SYN all-vs-all N={args.genomes} P={args.prot} (BASELINE configs[2] DB; "
                                   + ("block-cyclic rows, RCCL send/recv into rank 0)" if cyclic else
                                      "row-block sharded, RCCL gather to rank 0)"),
                       "genomes": args.genomes, "proteins": args.prot, "pairs": n_pairs, "F": n_f,
                       "events": total_events, "events_per_s": round(total_events / (ms_per_step * 1e-3), 1),
                       "parallelism": f"rowcyclic{world}" if cyclic else f"rowblock{world}",
                       "gather_pipeline": {"chunks_per_step": nch, "buffer_sets": slots,
                                           "form": "grouped send/recv of row-group segments" if cyclic
                                           else "gather of row blocks"},
                       "hot_path_GBps": round(step_bytes / (ms_per_step * 1e-3) / 1e9, 1),
                       "k_rows_ms_max_rank": round(k_rows_ms_max, 4),
                       "k_build_ms_max_rank": round(k_build_ms_max, 4)},
            "roofline": roofline,
            "load": load,
            "cpu_baseline": cpu,
        }
        if rehearse:
            line["rehearsal"] = "gloo, all ranks on one GPU, gather through host memory: flow check, not a measurement"
        if one_gpu:
            line["rehearsal"] = ("RCCL (nccl backend), all ranks on one GPU as separate NCCL hosts, transfers over "
                                 "RCCL's socket transport on loopback: the RCCL path executes; not a measurement")
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
