#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 bf16 image-classification stream, micro-batched.

Metric (BASELINE.json): whole-node records/sec + p50 per-record latency, ResNet-50 stream,
DP = number of GPUs (one process per GPU; launched by torch.distributed.run for N > 1).

Each rank runs the framework's streaming inference path on its own GPU:

  synthetic record source (decoded uint8 256x256x3 images, one record per image)
    → MicroBatcher (max_batch = --batch)
    → PipelinedGpuRunner: C++ gather into pinned slot → H2D on a side stream →
      hipGraph replay of the compiled ResNet-50 plan (fused resize+normalize kernel,
      29 implicit-GEMM MFMA convs with folded BN / fused residual+ReLU, pool, FC GEMM,
      fused softmax+top-5) → D2H of top-5 labels/probabilities
    → sink (per-record latency = result on host − record ingest)

Weights: random init (no network); rank 0's compiled weights are RCCL-broadcast to every
other rank (the DP model-distribution path).  A "step" is one micro-batch of --batch
records per GPU (weak scaling).  W warmup steps, then exactly K timed steps bracketed by a
barrier + device synchronize; the elapsed time is the MAX over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "records/sec (whole node) + p50 per-record latency, ResNet-50 stream DP=1/8"
METRIC_BERT = "records/sec (whole node) + p50 per-record latency, BERT-base text-classification stream"
METRIC_INCEPTION = "records/sec (whole node) + p50 per-record latency, Inception-v3 fp8 image stream"


def self_launch(args) -> int | None:
    """``--gpus N`` (N > 1) outside a launcher: start N ranks ourselves, one per GPU.

    The reference's data parallelism is operator parallelism — every subtask opens its own
    model (``inception.scala:21-22``, ``DefaultSavedModelLoader.scala:40-56``); here a
    subtask is a process bound to one GPU.  This parent never touches HIP (it does not
    even import torch: GPUs are counted from the KFD topology in sysfs,
    ``utils/gpus.py``): it checks that N GPUs are visible, runs ``torch.distributed.run`` as a CHILD process with
    the same arguments (the ranks then see WORLD_SIZE and take the normal path, exactly as
    under the driver's own torchrun) and exits with the child's status; rank 0's JSON line
    reaches our stdout unchanged.  Returns None when no launch is needed."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import socket
    import subprocess

    if not args.rehearse_fake_comm:
        from flink_tensorflow_amd.utils.gpus import sysfs_gpu_count

        n = sysfs_gpu_count()
        if n < args.gpus:
            print(f"[bench] --gpus {args.gpus} but {n} GPU(s) visible: refusing (no silent fallback to fewer "
                  "ranks)", file=sys.stderr)
            return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    return subprocess.call(cmd, env=env)


def run_launch_check(args, comm, rank, ws):
    """Rendezvous + one object exchange; rank 0 prints the world every rank reported."""
    import torch

    seen = comm.all_gather_object({"rank": rank, "world": ws, "pid": os.getpid(),
                                   "local_rank": int(os.environ.get("LOCAL_RANK", 0)),
                                   "gpus_visible": torch.cuda.device_count()})
    comm.barrier()
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": args.gpus, "world_size": ws,
                          "comm_world_size": comm.rank_size()[1], "ranks": [s["rank"] for s in seen],
                          "pids_distinct": len({s["pid"] for s in seen}) == ws,
                          "communicator": type(comm.get()).__name__ if comm.is_dist() else None}), flush=True)
    comm.destroy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="micro-batch (records per GPU per step)")
    ap.add_argument("--image-hw", type=int, default=None,
                    help="decoded source image size (resnet50: 256 resized to 224; inception_v3: 299)")
    ap.add_argument("--depth", type=int, default=3, help="pipeline slots")
    ap.add_argument("--gather-threads", type=int, default=8, help="native copy threads staging a micro-batch")
    ap.add_argument("--lane-offset-us", type=float, default=1500.0,
                    help="when the pipeline starts from empty, delay the k-th lane's first batch by k x this "
                         "(a stream-ordered delay kernel): the lanes start in the staggered phase of the steady "
                         "state instead of in step (profiles/r05_u: ResNet-50's first two batches 6.95 ms "
                         "instead of 7.3 / 8.1; 0 = off)")
    ap.add_argument("--no-numa", action="store_true", help="do not pin this rank to its GPU's NUMA node")
    ap.add_argument("--no-graph", action="store_true", help="disable hipGraph capture")
    ap.add_argument("--no-gc-freeze", action="store_true",
                    help="leave the setup objects to the cyclic GC (A/B of the runner's gc.freeze)")
    ap.add_argument("--pool", type=int, default=512, help="distinct synthetic records cycled by the source")
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "bert", "bert_graph", "widedeep",
                                                           "inception_v3"],
                    help="resnet50 = BASELINE headline; bert = BERT-base text-classification stream; "
                         "widedeep = Wide&Deep online training (DP gradient all-reduce); "
                         "inception_v3 = fp8 Inception-v3 stream with bucketed dynamic batching; bert_graph = "
                         "the BERT-base classifier as a TF GraphDef (modeling.py layout) through the graph "
                         "compiler (token-packed unless --no-pack)")
    ap.add_argument("--seq-len", type=int, default=128)
    ap.add_argument("--token-granule", type=int, default=2048,
                    help="bert_graph: token-capacity step of the packed plans (0: graph/packed.default_granule)")
    ap.add_argument("--precision", default=None, choices=["bf16", "fp8"],
                    help="compute precision of the compiled CNN plan (inception_v3 default fp8)")
    ap.add_argument("--buckets", default=None,
                    help="comma-separated extra batch buckets compiled next to --batch; with --dynamic the "
                         "per-step batch size varies and each micro-batch runs on the smallest bucket")
    ap.add_argument("--dynamic", action="store_true", help="variable micro-batch sizes (uniform in [B/4, B])")
    ap.add_argument("--bucket-step", type=int, default=8,
                    help="with --dynamic (and no --buckets): a compiled bucket every this many records from "
                         "B/4 to B (padding to the bucket is the cost of dynamic sizes; plans share one arena)")
    ap.add_argument("--offered-rate", type=float, default=None,
                    help="open-loop latency mode: records ARRIVE at this rate (records/s per GPU, Poisson); "
                         "each is stamped at its arrival, micro-batches form in a MicroBatcher (--batch, "
                         "--max-delay-ms) and p50/p99 are arrival -> result on host.  Runs --steps x --batch "
                         "arrivals after --warmup x --batch warm-up arrivals")
    ap.add_argument("--max-delay-ms", type=float, default=2.0, help="MicroBatcher deadline (offered-rate mode)")
    ap.add_argument("--no-pack", action="store_true", help="bert / bert_graph: run padded batches (no token packing)")
    ap.add_argument("--rehearse-fake-comm", action="store_true",
                    help="REHEARSAL ONLY: several ranks on one GPU exchange through the test loopback "
                         "communicator (host-staged) instead of RCCL, to exercise the multi-rank control flow "
                         "of this script where there is one GPU; numbers from such runs are not results")
    ap.add_argument("--lanes", type=int, default=None,
                    help="compute lanes: independent plan instances on their own HIP streams, batches round-robin "
                         "(default: 3 for inception_v3, 2 otherwise; measured in profiles/r01_lanes, r05_m, "
                         "r06_lanes: Inception-v3 fp8 +3.7 %% static / +7.6 %% dynamic at 3, -12 %% at 4; "
                         "ResNet-50 -2 %% at 3; BERT-base +0.4 %% and p50 26.5 -> 20.5 ms at 2 instead of 3)")
    ap.add_argument("--no-interleave", action="store_true",
                    help="A/B: launch a batch's per-piece head kernels after the whole host gather instead of "
                         "interleaved with it")
    ap.add_argument("--timeline", action="store_true",
                    help="also print, per timed batch, its lane and the GPU times of its first H2D piece, first "
                         "kernel and completion relative to the start of the timed window (diagnostics)")
    ap.add_argument("--job", action="store_true",
                    help="JOB MODE (resnet50, inception_v3, bert_graph, widedeep): ONE DataStream job with --gpus "
                         "worker-process subtasks, one GPU "
                         "each — a source chained into each subtask's worker, the ResNet-50 operator with "
                         "distributed_weights (rank 0 compiles, weights broadcast over the operator's RCCL "
                         "group) — timed on the operator (batching/timed.py).  Run as ONE process (not under "
                         "torch.distributed.run): the job starts its own workers")
    ap.add_argument("--wd-steps-per-round", type=int, default=8,
                    help="widedeep --job: full micro-batches a trainer subtask gathers before it calls an agreement "
                         "round (each round runs all of them as agreed steps)")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, rendezvous, exchange one object per rank and print the world the "
                         "communicator sees (no model; with --rehearse-fake-comm it runs on a CPU-only box)")
    args = ap.parse_args()

    if args.job:
        return run_job(args)
    rc = self_launch(args)
    if rc is not None:
        raise SystemExit(rc)

    import torch

    from flink_tensorflow_amd.batching.engine import PipelinedGpuRunner
    from flink_tensorflow_amd.graph.compiler import CompiledFunction
    from flink_tensorflow_amd.graph.graph import Graph
    from flink_tensorflow_amd.models.zoo.resnet import resnet50_flops_per_image, resnet50_graph_def
    from flink_tensorflow_amd.parallel import comm
    from flink_tensorflow_amd.utils.metrics import MetricGroup

    if args.rehearse_fake_comm:
        from flink_tensorflow_amd.parallel.fake import FakeCommunicator

        comm.init_distributed(communicator=FakeCommunicator,
                              device=f"cuda:{comm.local_device(comm.world()[2])}" if comm.gpu_count() else "cpu")
    else:
        comm.init_distributed()
    rank, ws, local = comm.world()
    if ws != args.gpus:  # never report a different world than the one asked for
        raise SystemExit(f"[bench] --gpus {args.gpus} but WORLD_SIZE={ws}: refusing to measure another world size")
    if comm.rank_size()[1] != ws:
        raise SystemExit(f"[bench] communicator holds {comm.rank_size()[1]} ranks, WORLD_SIZE={ws}")
    if args.launch_check:
        return run_launch_check(args, comm, rank, ws)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    if not args.rehearse_fake_comm and comm.gpu_count() < ws:
        raise SystemExit(f"[bench] WORLD_SIZE={ws} but only {comm.gpu_count()} GPU(s) visible to rank {rank}")
    dev = torch.device("cuda", comm.local_device(local))
    torch.cuda.set_device(dev)
    # stage records on the GPU's socket (every rank, DP=1 included): the gather threads and
    # the pinned slots they write are first-touched there
    numa = comm.bind_to_gpu_numa(dev) if not args.no_numa else None

    if args.model == "widedeep":
        return run_widedeep(args, dev, rank, ws)
    B = args.batch
    HW = args.image_hw or (299 if args.model == "inception_v3" else 256)
    precision = args.precision or ("fp8" if args.model == "inception_v3" else "bf16")
    t0 = time.perf_counter()
    from flink_tensorflow_amd.batching.arena import DeviceArena
    from flink_tensorflow_amd.config import EngineConfig

    lanes = args.lanes or (3 if args.model == "inception_v3" else 2)
    budget = EngineConfig().arena_bytes(dev) // lanes  # this subtask's HBM share, split over its lanes
    lane_plans, params = [], []
    if args.model == "inception_v3":
        from flink_tensorflow_amd.models.zoo.inception_v3 import inception_v3_flops_per_image, inception_v3_graph_def

        graph = Graph.from_graph_def(inception_v3_graph_def(image_hw=(HW, HW), top_k=5, seed=0))
        sizes = sorted({B} | {int(b) for b in (args.buckets or "").split(",") if b}
                       | (set(range(max(args.bucket_step, B // 4), B, args.bucket_step))
                          if args.dynamic and not args.buckets else set()))
        rng = np.random.default_rng(1234 + rank)
        pool = rng.integers(0, 256, size=(args.pool, HW, HW, 3), dtype=np.uint8)
        calib = torch.from_numpy(pool[: min(64, args.pool)])
        for lane in range(lanes):
            arena = DeviceArena(dev, budget, name=f"rank{rank}/lane{lane}")
            plans = {}
            for b in sorted(sizes, reverse=True):  # one captured plan per bucket, largest first: one shared slab
                cb = {"images:0": calib[:b] if b <= calib.shape[0] else calib.repeat((b + 63) // 64, 1, 1, 1)[:b]}
                plans[b] = CompiledFunction(graph, {"images:0": ((b, HW, HW, 3), "UINT8")}, ["top_k:0", "top_k:1"],
                                            dev, use_graph=not args.no_graph, strict=True, precision=precision,
                                            calibration=cb if precision == "fp8" else None, arena=arena)
            lane_plans.append(plans)
            params += [t for p in plans.values() for t in p.params]
        feed, rec_shape, rec_dtype = "images:0", (HW, HW, 3), torch.uint8
        flops_per_record = inception_v3_flops_per_image(299)
        model_name = "Inception-v3"
        data = f"synthetic decoded uint8 {HW}x{HW}x3 images, random-init weights, fp8 scales calibrated on them"
        seq = None
    elif args.model == "resnet50":
        gd = resnet50_graph_def(image_hw=(HW, HW), top_k=5, seed=0)
        graph = Graph.from_graph_def(gd)
        sizes = sorted({B} | {int(b) for b in (args.buckets or "").split(",") if b}
                       | (set(range(max(args.bucket_step, B // 4), B, args.bucket_step))
                          if args.dynamic and not args.buckets else set()))
        for lane in range(lanes):
            arena = DeviceArena(dev, budget, name=f"rank{rank}/lane{lane}")
            plans = {}
            for b in sorted(sizes, reverse=True):  # largest first: every bucket plan shares one slab
                plans[b] = CompiledFunction(graph, {"images:0": ((b, HW, HW, 3), "UINT8")}, ["top_k:0", "top_k:1"],
                                            dev, use_graph=not args.no_graph, strict=True, precision=precision,
                                            arena=arena)
            lane_plans.append(plans)
            params += [t for p in plans.values() for t in p.params]
        feed, rec_shape, rec_dtype = "images:0", (HW, HW, 3), torch.uint8
        flops_per_record = resnet50_flops_per_image(224)
        rng = np.random.default_rng(1234 + rank)
        pool = rng.integers(0, 256, size=(args.pool, HW, HW, 3), dtype=np.uint8)
        model_name, data = "ResNet-50 v1.5", f"synthetic decoded uint8 {HW}x{HW}x3 images, random-init weights"
        seq = None
    elif args.model == "bert_graph":
        from flink_tensorflow_amd.models.zoo.bert import BertConfig
        from flink_tensorflow_amd.models.zoo.bert_graph import bert_graph_def

        cfg = BertConfig.base()
        seq = args.seq_len
        gd, _ = bert_graph_def(cfg, seq, seed=rank, mask_from_ids=True)
        graph = Graph.from_graph_def(gd)
        for lane in range(lanes):
            arena = DeviceArena(dev, budget, name=f"rank{rank}/lane{lane}")
            if args.no_pack:
                p = CompiledFunction(graph, {"input_ids:0": ((B, seq), "INT32")}, ["logits:0"], dev,
                                     use_graph=not args.no_graph, strict=True, arena=arena)
            else:  # padding-free: one plan per token capacity, picked per micro-batch on the host
                from flink_tensorflow_amd.graph.packed import PackedFunction, default_granule

                p = PackedFunction(graph, {"input_ids:0": ((B, seq), "INT32")}, ["logits:0"], dev,
                                   use_graph=not args.no_graph, strict=True, arena=arena,
                                   granule=args.token_granule or default_granule(B, seq))
            lane_plans.append({B: p})
            params += p.params
        feed, rec_shape, rec_dtype = "input_ids:0", (seq,), torch.int32
        rng = np.random.default_rng(1234 + rank)
        pool = rng.integers(1000, cfg.vocab_size, size=(args.pool, seq), dtype=np.int32)
        lens = rng.integers(seq // 2, seq + 1, size=args.pool)
        for i, n in enumerate(lens):
            pool[i, n:] = 0
        pool[:, 0] = 101
        h, it = cfg.hidden, cfg.intermediate
        L = lens if not args.no_pack else np.full(args.pool, seq)  # useful work: real tokens only
        flops_per_record = float(np.mean(2.0 * L * cfg.layers * (4 * h * h + 2 * h * it)
                                         + 4.0 * L * L * h * cfg.layers))
        model_name = "BERT-base (seq classification), TF GraphDef through the graph compiler"
        data = (f"synthetic token ids, seq {seq} (real lengths U[{seq // 2},{seq}]), random-init weights, "
                + ("padded execution" if args.no_pack else "padding-free (token-packed) compiled plans"))
    else:
        from flink_tensorflow_amd.models.zoo.bert import (BertConfig, BertDeviceWeights, BertEncoderPlan,
                                                          PackedBertEncoder, init_bert_weights)

        cfg = BertConfig.base()
        seq = args.seq_len
        w = BertDeviceWeights(init_bert_weights(cfg, seed=rank), cfg, dev)  # rank-local init, then broadcast
        for lane in range(lanes):  # lanes share the weights, each has its own activation buffers
            if args.no_pack:
                p = BertEncoderPlan(w, B, seq, use_graph=not args.no_graph)
            else:  # padding-free: each micro-batch runs on the token capacity of its real tokens
                p = PackedBertEncoder(w, B, seq, use_graph=not args.no_graph)
            lane_plans.append({B: p})
        params = w.tensors()
        feed, rec_shape, rec_dtype = "ids", (seq,), torch.int32
        rng = np.random.default_rng(1234 + rank)
        pool = rng.integers(1000, cfg.vocab_size, size=(args.pool, seq), dtype=np.int32)
        lens = rng.integers(seq // 2, seq + 1, size=args.pool)
        for i, n in enumerate(lens):
            pool[i, n:] = 0
        pool[:, 0] = 101
        # useful work: the real tokens of the records (padding rows are not counted as FLOPs)
        flops_per_record = lane_plans[0][B].flops(lens) / len(lens)
        model_name = "BERT-base (seq classification)"
        data = (f"synthetic token ids, seq {seq} (real lengths U[{seq // 2},{seq}]), random-init weights, "
                + ("padded execution" if args.no_pack else "padding-free (packed) execution"))
    plan = lane_plans[0][B]
    params = list({t.data_ptr(): t for t in params}.values())  # interned / shared: each storage once
    # rank 0's weights to all ranks over RCCL (one flattened buffer per dtype); in place,
    # so the captured hipGraphs stay valid
    torch.cuda.synchronize(dev)
    comm.barrier()
    tb = time.perf_counter()
    nbytes = comm.broadcast_tensors(params, src=0)
    torch.cuda.synchronize(dev)
    bcast_s = time.perf_counter() - tb
    compile_s = time.perf_counter() - t0

    records = [pool[i] for i in range(args.pool)]
    runner = PipelinedGpuRunner(lane_plans, feed, lambda p: p.output_tensors(), rec_shape, rec_dtype,
                                depth=args.depth, device=dev, gather_threads=args.gather_threads,
                                lane_offset_us=args.lane_offset_us, freeze_gc=not args.no_gc_freeze,
                                timeline=args.timeline, interleave_head=not args.no_interleave)

    if args.offered_rate:
        return run_offered(args, runner, records, B, rank, ws, dev, comm, MetricGroup, model_name, data, lanes,
                           sorted(lane_plans[0]))

    cursor = 0
    lat = []
    n_done = 0
    n_sub = 0
    size_rng = np.random.default_rng(99)

    def step(collect):
        nonlocal cursor, n_done, n_sub
        n = int(size_rng.integers(max(1, B // 4), B + 1)) if args.dynamic else B
        batch = [records[(cursor + i) % args.pool] for i in range(n)]
        cursor += n
        if collect:
            n_sub += n
        # closed loop: a record "arrives" when the source hands it over, i.e. right here,
        # before staging (the open-loop --offered-rate mode measures arrival -> result
        # under a rate-limited source, including batch-formation wait)
        now = time.perf_counter()
        ts = np.full(n, now)
        for r in runner.poll() + runner.submit(batch, ts):
            n_done += r.n
            if collect:
                lat.append(r.latencies[: r.n])

    for _ in range(args.warmup):
        step(False)
    for r in runner.drain():
        pass
    torch.cuda.synchronize(dev)
    comm.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    runner.mark()
    for _ in range(args.steps):
        step(True)
    for r in runner.drain():
        lat.append(r.latencies[: r.n])
    torch.cuda.synchronize(dev)
    comm.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    elapsed_max = comm.all_reduce_scalar(elapsed, "max", device=dev)

    lat_all = np.concatenate(lat) if lat else np.zeros(1)
    # node-level percentiles: per-rank latency histograms merged bucket-wise (one all-reduce)
    mg = MetricGroup("bench")
    mg.histogram("latency_s").update_many(lat_all)
    node_lat = comm.allgather_metrics(mg)["histograms"]["latency_s"]
    n_rec = n_sub if args.dynamic else B * args.steps
    per_gpu = n_rec / elapsed
    total = comm.all_reduce_scalar(float(n_rec), "sum", device=dev) / elapsed_max
    per_rank = comm.all_gather_object(round(per_gpu, 1))
    flops = flops_per_record * total
    if rank == 0:
        out = {
            "metric": {"resnet50": METRIC, "bert": METRIC_BERT, "bert_graph": METRIC_BERT,
                       "inception_v3": METRIC_INCEPTION}[args.model],
            "value": round(total, 1),
            "unit": "records/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp8 (e4m3 weights+activations, fp32 accumulate)" if precision == "fp8" else "bf16",
            "data": data,
            "config": {"model": model_name, "global_batch": B * ws, "seq_len": seq,
                       "parallelism": f"dp{ws}", "micro_batch_per_gpu": B,
                       "input_hw": (299 if args.model == "inception_v3" else 224) if seq is None else None,
                       "batch_buckets": sorted(lane_plans[0]), "dynamic_batching": args.dynamic,
                       "compute_lanes": lanes, "lane_offset_us": args.lane_offset_us},
            "p50_latency_ms": round(node_lat["p50"] * 1e3, 3),
            "p99_latency_ms": round(node_lat["p99"] * 1e3, 3),
            "per_gpu_records_per_s": round(per_gpu, 1),
            "per_rank_records_per_s": per_rank,
            "comm_world_size": comm.rank_size()[1],
            "model_tflops_per_s": round(flops / 1e12, 1),
            "compile_s": round(compile_s, 2),
            "weights_broadcast_bytes": nbytes,
            "weights_broadcast_s": round(bcast_s, 4),
            "plan": plan.summary() if hasattr(plan, "summary") else {"hip_graph": plan.graph is not None},
            "arena": arena.stats() if args.model not in ("bert",) else None,
            "numa_binding_rank0": numa,
            "host_ms_per_batch": {k: round(v * 1e3 / max(1, runner.batches), 3) for k, v in runner.host_s.items()},
        }
        print(json.dumps(out), flush=True)
        if runner.timeline is not None:
            print(json.dumps({"timeline": runner.timeline, "elapsed_ms": round(elapsed * 1e3, 3)}), flush=True)
    comm.destroy()


def run_job(args):
    """``--job``: the headline config as the framework's own job model.
    This process is the coordinator: it never touches HIP; each subtask's worker process
    binds its GPU, joins the operator's communicator (RCCL), compiles (rank 0's weights
    are broadcast), generates its synthetic records in place (source chained into the
    worker: no record crosses a process boundary) and runs W + K micro-batches; the
    operator times the K (barrier + synchronize on both sides) and the JSON line reports
    the max elapsed over subtasks."""
    import shutil
    import tempfile

    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
        raise SystemExit("[bench] --job runs one coordinator process; do not launch it under torch.distributed.run")
    from flink_tensorflow_amd.utils.gpus import sysfs_gpu_count

    if sysfs_gpu_count() < args.gpus:
        raise SystemExit(f"[bench] --job --gpus {args.gpus} but {sysfs_gpu_count()} GPU(s) visible")
    if args.model == "widedeep":
        return run_job_widedeep(args)
    if args.model not in ("resnet50", "inception_v3", "bert_graph"):
        raise SystemExit("[bench] --job: resnet50, inception_v3, bert_graph or widedeep")
    from flink_tensorflow_amd.batching.timed import TimedWindow
    from flink_tensorflow_amd.runtime import StreamExecutionEnvironment
    from flink_tensorflow_amd.runtime.sources import DiscardingSink

    B, W, K, P = args.batch, args.warmup, args.steps, args.gpus
    pool_n = args.pool
    out_dir = tempfile.mkdtemp(prefix="ftm-bench-job-")
    t0 = time.perf_counter()
    seq = None
    try:
        if args.model in ("resnet50", "inception_v3"):
            from flink_tensorflow_amd.models.zoo.image_classifier import InceptionV3Model, ResNet50Model

            inc = args.model == "inception_v3"
            HW = args.image_hw or (299 if inc else 256)
            lanes = args.lanes or (3 if inc else 2)
            base = InceptionV3Model if inc else ResNet50Model

            class JobModel(TimedWindow, base):
                pass

            extra = {}
            if inc:  # one calibration set for every subtask: the same fp8 scales on every rank
                extra["calibration_images"] = np.random.default_rng(1234).integers(0, 256, size=(64, HW, HW, 3),
                                                                                   dtype=np.uint8)
            model = JobModel(image_hw=(HW, HW), buckets=(B,), distributed_weights=True, lanes=lanes,
                             depth=args.depth, lane_offset_us=args.lane_offset_us, **extra)

            def records(idx, par, start):  # runs in the subtask's worker process
                pool = np.random.default_rng(1234 + idx).integers(0, 256, size=(pool_n, HW, HW, 3), dtype=np.uint8)
                for i in range(start, (W + K) * B, 64):  # bulk: runs of 64 records per hand-over
                    yield [pool[(i + k) % pool_n] for k in range(min(64, (W + K) * B - i))]

            if inc:
                from flink_tensorflow_amd.models.zoo.inception_v3 import inception_v3_flops_per_image

                metric, name, flops = METRIC_INCEPTION, "Inception-v3", inception_v3_flops_per_image(299)
                dtype = "fp8 (e4m3 weights+activations, fp32 accumulate)"
            else:
                from flink_tensorflow_amd.models.zoo.resnet import resnet50_flops_per_image

                metric, name, flops, dtype = METRIC, "ResNet-50 v1.5", resnet50_flops_per_image(224), "bf16"
            data = f"synthetic decoded uint8 {HW}x{HW}x3 images generated in each worker, random-init weights"
            input_hw = 299 if inc else 224
        else:  # the BERT-base classifier as a TF SavedModel (modeling.py GraphDef, weights as variables)
            from flink_tensorflow_amd.models.batched import SignatureBatchedModel
            from flink_tensorflow_amd.models.zoo.bert import BertConfig
            from flink_tensorflow_amd.models.zoo.bert_graph import export_bert_saved_model

            class JobModel(TimedWindow, SignatureBatchedModel):
                pass

            cfg = BertConfig.base()
            seq = args.seq_len
            lanes = args.lanes or 2
            sm = export_bert_saved_model(os.path.join(out_dir, "bert_savedmodel"), cfg, seq, seed=0,
                                         mask_from_ids=True)
            model = JobModel(sm, output_keys=["logits"], buckets=(B,), lanes=lanes, depth=args.depth,
                             distributed_weights=True, lane_offset_us=args.lane_offset_us)
            vocab = cfg.vocab_size

            def records(idx, par, start):
                rng = np.random.default_rng(1234 + idx)
                pool = rng.integers(1000, vocab, size=(pool_n, seq), dtype=np.int32)
                lens = rng.integers(seq // 2, seq + 1, size=pool_n)
                for i, n in enumerate(lens):
                    pool[i, n:] = 0
                pool[:, 0] = 101
                for i in range(start, (W + K) * B, 64):
                    yield [pool[(i + k) % pool_n] for k in range(min(64, (W + K) * B - i))]

            metric, name, flops, dtype = METRIC_BERT, "BERT-base (seq classification), TF SavedModel", None, "bf16"
            data = (f"synthetic token ids generated in each worker, seq {seq} (real lengths U[{seq // 2},{seq}]), "
                    "random-init weights, padding-free (token-packed) compiled plans")
            input_hw = None
        model.timed_window(W, K, os.path.join(out_dir, "ranks"))
        env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(P)
        env.enable_job_communicator(True)  # one RCCL group for the operator, P = 1 included
        src = env.generate(records, bulk=True).run_in_processes()
        src.map_with_model_batched(model, None, max_batch=B, max_delay_ms=60_000.0, name=args.model) \
            .run_in_processes().add_sink(DiscardingSink()).run_in_processes()  # results stay in the worker
        res = env.execute("bench-job")
        wall = time.perf_counter() - t0
        ranks = []
        for r in range(P):
            with open(os.path.join(out_dir, "ranks", f"rank{r}.json")) as f:
                ranks.append(json.load(f))
    finally:
        shutil.rmtree(out_dir, ignore_errors=True)
    elapsed = max(r["elapsed_s"] for r in ranks)
    n_rec = sum(r["records"] for r in ranks)
    lat = np.concatenate([np.asarray(r["latencies_s"]) for r in ranks]) if ranks else np.zeros(1)
    total = n_rec / elapsed
    print(json.dumps({
        "metric": metric, "value": round(total, 1), "unit": "records/s", "n_gpus": P, "steps": K, "warmup": W,
        "ms_per_step": round(elapsed / K * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": dtype, "data": data,
        "config": {"model": name, "global_batch": B * P, "seq_len": seq, "parallelism": f"dp{P}",
                   "micro_batch_per_gpu": B, "input_hw": input_hw, "batch_buckets": [B], "compute_lanes": lanes,
                   "lane_offset_us": args.lane_offset_us,
                   "mode": "job: one DataStream job, P worker-process GPU subtasks, chained sources, "
                           "distributed_weights over the operator's communicator"},
        "p50_latency_ms": round(float(np.percentile(lat, 50)) * 1e3, 3) if lat.size else None,
        "p99_latency_ms": round(float(np.percentile(lat, 99)) * 1e3, 3) if lat.size else None,
        "per_rank_records_per_s": [round(r["records"] / r["elapsed_s"], 1) for r in ranks],
        "communicator": ranks[0]["communicator"], "comm_world_size": ranks[0]["world"],
        "host_ms_per_batch_rank0": ranks[0].get("host_ms_per_batch"), "plan": ranks[0].get("plan"),
        "model_tflops_per_s": round(flops * total / 1e12, 1) if flops else None,
        "job_wall_s": round(wall, 2), "job_attempts": res.attempts}), flush=True)


def run_job_widedeep(args):
    """``--job --model widedeep``: Wide&Deep online training as ONE DataStream job
    (VERDICT r5 #2): P worker-process subtasks of a ``LockstepTrainer`` (the agreed-step
    co-process trainer, one GPU each), each fed by a generator source chained into its
    worker that hands over blocks of packed 192-B click rows.  Every agreed step is the
    captured fused step (pieces padded to the micro-batch, ``{nvalid, norm}`` in device
    memory); rounds carry up to ``--wd-steps-per-round`` full batches and agree over the
    host control channel.  The trainer times W + K agreed steps (``batching/timed.py``
    ``TimedSteps``); the JSON line reports the max elapsed over subtasks."""
    import shutil
    import tempfile

    from flink_tensorflow_amd.batching.timed import TimedSteps
    from flink_tensorflow_amd.models.zoo.wide_deep import (WideDeepConfig, WideDeepTrainer, pack_click_records,
                                                           synthetic_click_records)
    from flink_tensorflow_amd.runtime import RestartStrategy, StreamExecutionEnvironment
    from flink_tensorflow_amd.runtime.lockstep import LockstepTrainer
    from flink_tensorflow_amd.runtime.sources import DiscardingSink

    class JobTrainer(TimedSteps, LockstepTrainer):
        pass

    B = args.batch if args.batch != 256 else 4096
    W, K, P = args.warmup, args.steps, args.gpus
    spr = args.wd_steps_per_round
    blk = B  # rows per source block
    cfg = WideDeepConfig()
    out_dir = tempfile.mkdtemp(prefix="ftm-bench-wdjob-")
    if P > 1:  # the capturable fixed-capacity exchange; its overflow recovery is a job restart
        os.environ["FT_WD_SPARSE_EXCHANGE"] = "bucketed"
    t0 = time.perf_counter()
    try:
        env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(P)
        env.enable_job_communicator(P > 1)
        if P > 1:
            env.set_restart_strategy(RestartStrategy.fixed_delay(1, 0.0))
        total = (W + K) * B

        def clicks(idx, par, start):  # runs in the subtask's worker process
            pool = pack_click_records(synthetic_click_records(16 * B, cfg, seed=idx), cfg)
            i = start
            while i < total:
                o = i % len(pool)
                n = min(blk, total - i, len(pool) - o)
                yield pool[o:o + n]
                i += n

        trainer = JobTrainer(WideDeepTrainer(cfg, seed=0), B, max_delay_ms=20.0, steps_per_round=spr,
                             max_steps_per_round=max(spr, 64)).timed_window(W, K, out_dir)
        env.generate(clicks).run_in_processes().process(trainer, "widedeep-trainer").run_in_processes() \
            .add_sink(DiscardingSink()).run_in_processes()
        res = env.execute("bench-widedeep-job")
        wall = time.perf_counter() - t0
        ranks = []
        for r in range(P):
            with open(os.path.join(out_dir, f"rank{r}.json")) as f:
                ranks.append(json.load(f))
    finally:
        shutil.rmtree(out_dir, ignore_errors=True)
    elapsed = max(r["elapsed_s"] for r in ranks)
    n_rec = sum(r["records"] for r in ranks)
    value = n_rec / elapsed
    print(json.dumps({
        "metric": "records/sec (whole node), Wide&Deep online training (DP all-reduce)",
        "value": round(value, 1), "unit": "records/s", "n_gpus": P, "steps": K, "warmup": W,
        "ms_per_step": round(elapsed / K * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16 compute / fp32 master weights",
        "data": "synthetic Criteo-shaped click records as 192-B packed rows generated in each worker "
                "(source chained into the trainer), random init",
        "config": {"model": "Wide&Deep (26x100k x32 embeddings, MLP 1024-512-256)", "global_batch": B * P,
                   "seq_len": None, "parallelism": f"dp{P}", "micro_batch_per_gpu": B,
                   "mode": "job: one DataStream job, P worker-process LockstepTrainer subtasks, agreed steps "
                           "(host control channel), captured padded step",
                   "steps_per_round": spr},
        "per_rank_records_per_s": [round(r["records"] / r["elapsed_s"], 1) for r in ranks],
        "rounds": [r.get("rounds") for r in ranks], "job_wall_s": round(wall, 2),
        "job_attempts": res.attempts}), flush=True)


def run_offered(args, runner, records, B, rank, ws, dev, comm, MetricGroup, model_name, data, lanes, buckets):
    """Open-loop latency: Poisson arrivals at --offered-rate records/s per GPU.  Each record
    is stamped when it arrives (not when its batch is formed); a MicroBatcher forms
    micro-batches of up to --batch records or whatever arrived within --max-delay-ms; a
    batch of n runs on the smallest compiled bucket >= n.  Latency = arrival -> top-k on
    the host.  Reports achieved records/s and node-level p50/p99 (merged histograms)."""
    import torch

    from flink_tensorflow_amd.batching.engine import MicroBatcher

    rate = float(args.offered_rate)
    n_warm, n_meas = args.warmup * B, args.steps * B
    gaps = np.random.default_rng(7 + rank).exponential(1.0 / rate, n_warm + n_meas)
    batcher = MicroBatcher(B, args.max_delay_ms)
    lat, sizes = [], []

    def consume(done, measure_from):
        for r in done:
            keep = r.ingest_ts >= measure_from
            lat.append(r.latencies[: r.n][keep[: r.n]])

    def drive(n, measure_from):
        arrivals = time.perf_counter() + np.cumsum(gaps[:n])  # schedule relative to now
        i = 0
        while i < n or len(batcher):
            now = time.perf_counter()
            while i < n and arrivals[i] <= now:  # everything that has arrived by now
                b = batcher.add(records[i % len(records)], arrivals[i])  # stamped at ARRIVAL
                i += 1
                if b is not None:
                    sizes.append(len(b[0]))
                    consume(runner.submit(*b), measure_from)
            if batcher.due(now) or (i >= n and len(batcher)):
                b = batcher.flush()
                sizes.append(len(b[0]))
                consume(runner.submit(*b), measure_from)
            consume(runner.poll(), measure_from)
            if i < n and len(batcher) == 0:
                time.sleep(max(0.0, min(arrivals[i] - time.perf_counter(), 2e-4)))
        consume(runner.drain(), measure_from)

    drive(n_warm, float("inf"))
    lat.clear()
    sizes.clear()
    torch.cuda.synchronize(dev)
    comm.barrier()
    t0 = time.perf_counter()
    drive(n_meas, t0)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    comm.barrier()
    elapsed_max = comm.all_reduce_scalar(elapsed, "max", device=dev)
    mg = MetricGroup("bench")
    mg.histogram("latency_s").update_many(np.concatenate(lat) if lat else np.zeros(1))
    node_lat = comm.allgather_metrics(mg)["histograms"]["latency_s"]
    total = comm.all_reduce_scalar(float(n_meas), "sum", device=dev) / elapsed_max
    if rank == 0:
        print(json.dumps({
            "metric": f"p50/p99 arrival->result latency at an offered load, {model_name} stream",
            "value": round(node_lat["p50"] * 1e3, 3), "unit": "ms (p50)", "higher_is_better": False,
            "n_gpus": ws, "offered_records_per_s": round(rate * ws, 1), "achieved_records_per_s": round(total, 1),
            "p50_latency_ms": round(node_lat["p50"] * 1e3, 3), "p99_latency_ms": round(node_lat["p99"] * 1e3, 3),
            "max_batch": B, "max_delay_ms": args.max_delay_ms, "batch_buckets": buckets, "compute_lanes": lanes,
            "mean_batch": round(float(np.mean(sizes)), 1) if sizes else None, "batches": len(sizes),
            "records": n_meas, "dtype": "bf16", "data": data + "; Poisson arrivals"}), flush=True)
    comm.destroy()


def run_widedeep(args, dev, rank, ws):
    """Wide&Deep online training: a step = one micro-batch of --batch labelled click records
    per GPU, INCLUDING its collation: the records are fixed-size binary rows (label, 13
    dense, 26 categorical, 8 crossed ids = 192 B) gathered by the native stager into pinned
    memory, copied H2D and split on the device, then forward, backward with the bucketed
    RCCL all-reduce (+ row-sparse all-gather under DP), Adam + sparse Adagrad — the whole
    step replayed as one hipGraph (with the collectives inside it under DP)."""
    import torch

    from flink_tensorflow_amd.models.zoo.wide_deep import (PackedBatchStager, WideDeepConfig, WideDeepTrainer,
                                                           pack_click_records, synthetic_click_records)
    from flink_tensorflow_amd.parallel import comm

    B = args.batch if args.batch != 256 else 4096
    cfg = WideDeepConfig()
    t0 = time.perf_counter()
    if ws > 1 and "FT_WD_SPARSE_EXCHANGE" not in os.environ:
        import dataclasses

        from flink_tensorflow_amd import config as C

        # the capturable fixed-capacity exchange: a bounded run that checks for overflow at
        # its end (ex.check() below) and fails loudly, never a silent drop
        C.set_current(dataclasses.replace(C.current(), wd_sparse_exchange="bucketed"))
    tr = WideDeepTrainer(cfg, device=dev, seed=0)
    tr.open()
    pool_n = 16 * B
    rows = list(pack_click_records(synthetic_click_records(pool_n, cfg, seed=rank), cfg))
    stager = PackedBatchStager(cfg, B, dev)
    compile_s = time.perf_counter() - t0
    cursor = 0

    def step():
        nonlocal cursor
        batch = stager.stage(rows[cursor:cursor + B])
        cursor = (cursor + B) % pool_n
        return tr.train_step(batch=batch)

    if not args.no_graph:  # whole train step as one hipGraph (sync-free sparse path)
        try:
            tr.capture(stager.stage(rows[:B]))
        except RuntimeError as e:  # e.g. a collective library that cannot be stream-captured
            print(f"[bench] rank {rank}: whole-step capture failed ({e}); running the step eagerly",
                  file=sys.stderr)
            tr._graph = None
            torch.cuda.synchronize(dev)
    from flink_tensorflow_amd.utils.gcfreeze import freeze_setup_objects

    if not args.no_gc_freeze:
        freeze_setup_objects()  # as the pipelined runner does after its plans compile

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    comm.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    loss = None
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize(dev)
    comm.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    elapsed_max = comm.all_reduce_scalar(elapsed, "max", device=dev)
    total = ws * B * args.steps / elapsed_max
    ex = tr._exchange
    if ex is not None and hasattr(ex, "check"):
        ex.check()  # no bucket of the fixed-capacity exchange overflowed in the timed steps
    if rank == 0:
        print(json.dumps({
            "metric": "records/sec (whole node), Wide&Deep online training (DP all-reduce)",
            "value": round(total, 1), "unit": "records/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16 compute / fp32 master weights",
            "data": "synthetic Criteo-shaped click records (13 dense, 26 categorical, 8 crossed) as 192-B binary "
                    "rows, collated inside the timed step; random init",
            "config": {"model": "Wide&Deep (26x100k x32 embeddings, MLP 1024-512-256)", "global_batch": B * ws,
                       "seq_len": None, "parallelism": f"dp{ws}", "micro_batch_per_gpu": B},
            "final_loss": round(float(loss), 4), "setup_s": round(compile_s, 2),
            "hip_graph": tr._graph is not None,
            "sparse_exchange": type(ex).__name__ if ex is not None else ("allgather" if ws > 1 else None),
            "bucket_capacities": {str(k): v for k, v in getattr(ex, "_caps", {}).items()} or None}), flush=True)
    tr.close()
    comm.destroy()


if __name__ == "__main__":
    main()
