"""Benchmark of the IWAE hot path on MI355X (BASELINE.json metric:
"train images*k/sec and k=5000 test-NLL images/sec, 1-8 MI355X").

Workload (BASELINE.json configs[1], fits one GPU): IWAE, k=50, 2 stochastic
layers 784-200-200-100-100-50, batch 20 per GPU, one full train step (forward,
IWAE bound, backward, Adam) per step, device Philox noise, hipGraph replay.
Data: synthetic fixed-binarised 784-pixel images (MNIST-like pixel means,
mean ~0.13) resident in HBM; Glorot weights.  `value` = sample-rows (images*k)
per second over all ranks (weak scaling: 20 images per GPU, RCCL gradient
all-reduce for N > 1).  The k=5000 NLL over 10k synthetic images (configs[2],
sharded by image) is reported beside it under "nll", and the large-batch data-
parallel train step (configs[4]: B=4096 over 8 GPUs, i.e. 512 images per GPU,
k=50) under "large_batch" -- weak scaling at that per-GPU share.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...    (one process per GPU)

With --gpus N > 1 and no WORLD_SIZE in the environment, this process starts
the N ranks itself (torch.distributed.run as a child process, before any GPU
call here), relays rank 0's JSON line and exits with the workers' status.
Under the default backend (nccl = RCCL) N must not exceed the visible GPUs;
IWAE_DIST_BACKEND=gloo rehearses N ranks on one GPU.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HE, HD, LE, LD = [200, 100], [100, 200], [100, 50], [100, 784]
B_PER_GPU, K = 20, 50
LARGE_B_PER_GPU = 512              # configs[4]: global batch 4096 over 8 GPUs
# algorithmic train FLOP per image*sample, 2L k=50
TRAIN_FLOP_PER_ROW = 1_712_944
SAMPLE_ROW_MACS = 281_800          # per sample row, one pass over the sample-row Dense layers (2L)
NLL_FLOP_PER_IMAGE = 2.818e9
FP32_MFMA_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 spec peak
BF16_PEAK_TFLOPS = 2500.0          # MI355X_MICROARCH.md: BF16 MFMA dense peak
BF16X3_PEAK_TFLOPS = round(BF16_PEAK_TFLOPS / 3, 1)   # f32-accurate bf16x3 products: 3 bf16 MFMAs each
HBM_PEAK_GBS = 8000.0
# ---- roofline model: algorithmic FLOP and HBM bytes per launch
# of the train step's kernels, 2L model, from the layer widths.  Bytes count every
# tensor a launch must read or write across its boundary ONCE (f32, 4 B): the
# weights it multiplies, its inputs, and what a later launch reads; split-K
# partials, re-reads and padding are implementation traffic (the PMC "traffic"
# beside it shows them).  A kernel is MFMA-bound when its FLOP / byte ratio is
# above the ridge (833.3 TFLOP/s / 8 TB/s = 104 FLOP/B), else HBM-bound; frac =
# max(t_mfma, t_hbm) / t.
# (fin, fout, image rows?) per Dense layer: encoder layer 1 (per image), encoder
# layer 2, decoder prior layer, output MLP
LAYERS_2L = {"e1.l1": (784, 200, True), "e1.l2": (200, 200, True), "e1.head": (200, 200, True),
             "e2.l1": (100, 100, False), "e2.l2": (100, 100, False), "e2.head": (100, 100, False),
             "p.l1": (50, 100, False), "p.l2": (100, 100, False), "p.head": (100, 200, False),
             "o1": (100, 200, False), "o2": (200, 200, False), "o3": (200, 784, False)}
ROW_LAYERS = [k for k, v in LAYERS_2L.items() if not v[2]]
OUT_MLP, ENC_PRIOR = ["o1", "o2", "o3"], ["e2.l1", "e2.l2", "e2.head", "p.l1", "p.l2", "p.head"]
# floats per sample row the forward stores for later launches: h1, eps1; e2: y1, y2, (mu|zs), h2, eps2;
# prior: y1, y2, (mu|zs); output MLP: y1, y2, g; log q, log p, Bernoulli sum
FWD_STORE_ROW = 200 + (100 + 100 + 100 + 50 + 50) + (100 + 100 + 200) + (200 + 200 + 784) + 3
# output-MLP backward-data: reads g, dpx, y2, y1; writes dY2, dY1, dL/dh1
OUT_BWD_ROW = (784 + 1 + 200 + 200) + (200 + 200 + 100)
# encoder / prior backward-data: reads dlw; prior (mu|zs), its target h1, y2, y1; e2 (mu|zs), h2, eps2, y2,
# y1; writes prior dP, dY2, dY1, dL/dh1 (prior); e2 dP, dY2, dY1, dL/dh1 (encoder)
ENC_BWD_ROW = 1 + (200 + 100 + 100 + 100) + (100 + 50 + 50 + 100 + 100) + (200 + 100 + 100 + 100) + \
    (100 + 100 + 100 + 100)
# weight gradients of the sample-row layers: every X and dZ operand once (h1 feeds e2.l1 and o1: once), dpx
WGRAD_ROW = (100 + 100 + 100 + 50 + 100 + 100 + 200 + 200) + (100 + 100 + 100 + 100 + 100 + 200 + 200 + 200 + 784) + 1
# the first encoder layer's backward on image rows: reads per sample row h1, eps1, dlw and three dL/dh1
# sources; per image (mu|zs), y2, y1; writes per image dP0, dY2, dY1
IMG_BWD_ROW, IMG_BWD_IMG = 100 + 100 + 1 + 300, 200 + 200 + 200 + 600


def layer_params(names):
    return sum((LAYERS_2L[n][0] + 1) * LAYERS_2L[n][1] for n in names)


def layer_macs(names, bias=False):
    return sum((LAYERS_2L[n][0] + (1 if bias else 0)) * LAYERS_2L[n][1] for n in names)


N_PARAMS = layer_params(LAYERS_2L)


def kernel_work(kind, rows, images):
    """(algorithmic FLOP, algorithmic HBM bytes) of one launch of a train-step
    kernel kind over `rows` sample rows of `images` images (see above)."""
    W = 4.0 * layer_params(ROW_LAYERS)
    if kind == "fwd":          # sample-row forward: engine jobs E + O, or the ring kernel in train mode
        return 2.0 * rows * SAMPLE_ROW_MACS, W + 4.0 * (images * (784 + 200) + rows * FWD_STORE_ROW)
    if kind == "bwd":          # the engine's backward launch: jobs O' + E' (and the bound, a few KB)
        return 2.0 * rows * SAMPLE_ROW_MACS, W + 4.0 * rows * (OUT_BWD_ROW + ENC_BWD_ROW)
    if kind == "nrb":
        return 2.0 * rows * layer_macs(OUT_MLP), 4.0 * layer_params(OUT_MLP) + 4.0 * rows * OUT_BWD_ROW
    if kind == "nre":
        return 2.0 * rows * layer_macs(ENC_PRIOR), 4.0 * layer_params(ENC_PRIOR) + 4.0 * rows * ENC_BWD_ROW
    if kind == "dw":           # the sample-row layers' dW_aug = X_aug^T dZ, written once
        return 2.0 * rows * layer_macs(ROW_LAYERS, bias=True), 4.0 * (rows * WGRAD_ROW + layer_params(ROW_LAYERS))
    if kind == "img_bwd":      # job I': the first encoder layer's Gaussian backward (sum over k) + head^T, l2^T
        return (2.0 * images * (200 * 200 + 200 * 200),
                4.0 * (rows * IMG_BWD_ROW + images * IMG_BWD_IMG + layer_params(["e1.l2", "e1.head"])))
    if kind == "img_fwd":      # job I: the first encoder layer's l2 and head on image rows (after its input Dense)
        return (2.0 * images * (200 * 200 + 200 * 200),
                4.0 * (images * (200 + 200 + 200 + 200) + layer_params(["e1.l2", "e1.head"])))
    if kind == "tcu":          # job I' and the fused update in one launch (tcu_kernel)
        f1, b1 = kernel_work("img_bwd", rows, images)
        f2, b2 = kernel_work("upd", rows, images)
        return f1 + f2, b1 + b2
    if kind == "upd":          # every layer's dW + Adam (p, m, v read; p, m, v, g written) + FX / GX bf16 copies
        img_xz = images * (785 + 201 + 201 + 200 + 200 + 200)
        fl = 2.0 * (rows * layer_macs(ROW_LAYERS, bias=True) +
                    images * layer_macs(["e1.l1", "e1.l2", "e1.head"], bias=True))
        return fl, 4.0 * (rows * WGRAD_ROW + img_xz + 7 * N_PARAMS) + 8.0 * N_PARAMS
    raise ValueError(kind)


def roofline_of(flop, nbytes, us, peak_tflops=None, hbm_gbs=None):
    """Binding roofline of a launch: MFMA if flop / byte is above the ridge,
    else HBM; frac = max(t_mfma, t_hbm) / t."""
    pk = peak_tflops or round(2500.0 / 3, 1)
    hb = hbm_gbs or 8000.0
    t = us * 1e-6
    t_mfma, t_hbm = flop / (pk * 1e12), nbytes / (hb * 1e9)
    ai = flop / nbytes if nbytes else float("inf")
    if t_mfma >= t_hbm:
        return dict(bound="mfma", achieved=round(flop / t / 1e12, 3), peak=pk, unit="TFLOP/s",
                    frac=round(t_mfma / t, 4), flop_per_byte=round(ai, 1), ridge=round(pk * 1e3 / hb, 1),
                    alg_bytes=nbytes, flop=flop)
    return dict(bound="hbm", achieved=round(nbytes / t / 1e9, 1), peak=hb, unit="GB/s", frac=round(t_hbm / t, 4),
                flop_per_byte=round(ai, 1), ridge=round(pk * 1e3 / hb, 1), alg_bytes=nbytes, flop=flop)


LB_RECORD = "r06_large_batch_kernels.json"     # the large-batch step's committed kernel record
PMC_RECORD = "r06_pmc_traffic.json"            # the B = 20 step's committed per-launch HBM traffic (PMC)


PRECISION = ("fp32 values and fp32 accumulation everywhere; every sample-row matrix product of the train step "
             "(forward, backward-data and weight gradients) and of the NLL is a bf16x3 split product "
             "(a_hi b_hi + a_hi b_lo + a_lo b_hi on bf16 MFMA, ~2^-16 relative per product); the first encoder "
             "layer's input Dense (784 -> 200 on image rows) is exact f32 MFMA, at <= 32 images its l2 and head "
             "too (DESIGN.md section 4)")


def pixel_profile():
    """Fixed smooth MNIST-like per-pixel 'on' probability, mean ~0.13 (seed 0)."""
    rng = np.random.default_rng(0)
    yy, xx = np.mgrid[0:28, 0:28]
    r = np.sqrt((yy - 13.5) ** 2 + (xx - 13.5) ** 2)
    base = 0.355 * np.exp(-((r - 5.5) ** 2) / 18.0)
    pi = np.clip(base + 0.03 * rng.random((28, 28)), 0.0, 0.95).reshape(-1)
    return pi


def synthetic_images(n, seed):
    pi = pixel_profile()
    rng = np.random.default_rng(seed)
    return (rng.random((n, 784)) < pi).astype(np.float32), pi


CORES_NOTE = ("threads = the process's CPU affinity set capped by OMP_NUM_THREADS: the GPU pool gives each "
              "GPU a 16-CPU share of the host and sets OMP_NUM_THREADS=16 (nproc counts the whole machine); "
              "threads_curve shows how the oracle's small per-step BLAS calls scale with threads")


def host_cores():
    """(threads used, cores this process may run on, nproc): the threads are the
    cores of the process's CPU affinity set (the box's share), capped by
    OMP_NUM_THREADS when the environment sets it."""
    try:
        avail = len(os.sched_getaffinity(0))
    except Exception:          # pragma: no cover
        avail = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    used = min(avail, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else avail
    return used, avail, os.cpu_count() or 1


def _oracle_train_rate(O, seconds, threads, arch=None, k=None):
    """IWAE train steps of the oracle (B=20, k=50, 2L by default, float32, incl.
    the F:340 duplicate decoder pass) on `threads` BLAS threads for about `seconds`."""
    from threadpoolctl import threadpool_limits
    arch = arch or (HE, HD, LE, LD)
    k = k or K
    with threadpool_limits(limits=threads):
        spec = O.ModelSpec(*arch)
        x, pi = synthetic_images(B_PER_GPU, 1)
        rng = np.random.default_rng(2)
        params = O.cast_params(O.glorot_init(spec, rng, out_bias=O.output_bias_from_mean(pi)), np.float32)
        opt = O.Adam(1e-3, 0.9, 0.999, 1e-4)
        xf = x.astype(np.float32)
        steps, t0 = 0, time.perf_counter()
        while True:
            eps = O.draw_eps(spec, k, B_PER_GPU, rng, np.float32)
            J, g = O.objective_and_grads(params, spec, xf, eps, "IWAE", k, dup_decoder=True)
            flat = O.flatten_params(spec, params)
            new = opt.apply(flat, -O.flatten_params(spec, g).astype(np.float32))
            params = O.unflatten_params(spec, new, dtype=np.float32)
            steps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    return steps, el


def cpu_baseline(seconds=12.0):
    """The oracle (numpy restatement of the reference's op sequence, incl. the
    duplicate decoder pass at F:340) timed on host cores: IWAE train steps at
    the bench workload (B=20, k=50, 2L), float32.  `value` is the rate on the
    process's thread budget (`cores`); `threads_curve` is the rate at 1, 4 and
    that many threads (a third of the time each is spent on the curve)."""
    from oracle import iwae_oracle as O
    cores, avail, nproc = host_cores()
    curve = {}
    for t in sorted({1, min(4, cores)}):
        st, el = _oracle_train_rate(O, seconds / 6, t)
        curve[t] = round(st * B_PER_GPU * K / el, 1)
    steps, el = _oracle_train_rate(O, seconds * 2 / 3, cores)
    curve[cores] = round(steps * B_PER_GPU * K / el, 1)
    return dict(value=steps * B_PER_GPU * K / el, unit="image*samples/s", cores=cores, cores_available=avail,
                nproc=nproc, kind="port", threads_curve={str(k): v for k, v in sorted(curve.items())},
                cores_note=CORES_NOTE,
                sample=f"{steps} IWAE train steps (2L, k={K}, batch {B_PER_GPU}, float32 numpy, incl. the "
                       f"F:340 duplicate decoder pass) in {el:.1f} s on {cores} threads")


def cpu_baseline_configs0(seconds=4.0):
    """BASELINE configs[0] (experiment_example.py: IWAE k=5, 1 stochastic layer
    784-200-200-50, batch 20; the reference's TF CPU path): the oracle's train
    steps on the host cores, float32 -- the CPU figure beside configs0_train."""
    from oracle import iwae_oracle as O
    cores, avail, nproc = host_cores()
    _oracle_train_rate(O, 0.3, cores, arch=([200], [200], [50], [784]), k=5)      # warm-up (first BLAS calls)
    steps, el = _oracle_train_rate(O, seconds, cores, arch=([200], [200], [50], [784]), k=5)
    return dict(value=steps * B_PER_GPU * 5 / el, unit="image*samples/s", cores=cores, kind="port",
                sample=f"{steps} IWAE train steps (1L 784-200-200-50, k=5, batch {B_PER_GPU}, float32 numpy, incl. "
                       f"the F:340 duplicate decoder pass) in {el:.1f} s on {cores} threads")


def cpu_baseline_nll(seconds=8.0, k=5000):
    """the k=5000 NLL (get_NLL F:463 -> get_log_weights F:327-F:351,
    incl. the F:340 duplicate decoder pass) on the oracle, float32, on the host
    cores, over as many synthetic test images as fit in `seconds`; images/s
    extrapolates linearly to the 10k-image set (the path is per-image)."""
    from oracle import iwae_oracle as O
    try:
        from threadpoolctl import threadpool_limits
    except Exception:          # pragma: no cover
        threadpool_limits = None
    cores, avail, nproc = host_cores()
    ctx = threadpool_limits(limits=cores) if threadpool_limits else None
    try:
        spec = O.ModelSpec(HE, HD, LE, LD)
        xt, pi = synthetic_images(64, 99)
        rng = np.random.default_rng(2)
        params = O.cast_params(O.glorot_init(spec, rng, out_bias=O.output_bias_from_mean(pi)), np.float32)
        chunk = 1000
        n, t0 = 0, time.perf_counter()
        while n < xt.shape[0]:
            x = xt[n:n + 1].astype(np.float32)
            m_run, s_run = -np.inf, 0.0
            for s0 in range(0, k, chunk):
                e = O.draw_eps(spec, chunk, 1, rng, np.float32)
                lw = O.forward(params, spec, x, e, dup_decoder=True)["lw"].astype(np.float64)[:, 0]
                M = max(m_run, lw.max())
                s_run = s_run * math.exp(m_run - M) + np.exp(lw - M).sum()
                m_run = M
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    finally:
        if ctx is not None:
            ctx.__exit__(None, None, None)
    return dict(value=n / el, unit="images/s", cores=cores, cores_available=avail, nproc=nproc, kind="port",
                cores_note=CORES_NOTE, sample=f"{n} test images at k={k} (2L, float32 numpy, incl. the F:340 duplicate decoder pass) in "
                       f"{el:.1f} s; extrapolates linearly to 10k images")


def dist_backend():
    """nccl (= RCCL over xGMI) unless IWAE_DIST_BACKEND names another one (gloo:
    the one-GPU rehearsal of N ranks)."""
    return os.environ.get("IWAE_DIST_BACKEND", "nccl")


def visible_gpus():
    """GPUs this process may use.  torch.cuda.device_count() does not initialise
    the GPU on this image, so the launcher may call it before spawning ranks."""
    import torch
    return torch.cuda.device_count()


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(n, argv, port, script=None):
    """The child command that runs n ranks of this script on one node."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", script or os.path.abspath(__file__)] + list(argv)


def check_world(n, backend, ngpus):
    """A world of n ranks needs n GPUs under nccl (one process per GPU); gloo
    may place every rank on one GPU (rehearsal)."""
    if n < 1:
        raise SystemExit(f"--gpus must be >= 1, got {n}")
    if backend == "nccl" and n > ngpus:
        raise SystemExit(f"--gpus {n} needs {n} visible GPUs under nccl (RCCL, one process per GPU); "
                         f"{ngpus} visible. Set IWAE_DIST_BACKEND=gloo to rehearse {n} ranks on fewer GPUs.")


def launch_ranks(n, argv, script=None):
    """Run n ranks as a torch.distributed.run child (never an exec: this
    process has not touched the GPU and stays the parent); relay rank 0's
    JSON line to stdout, everything else to stderr; return the exit code."""
    check_world(n, dist_backend(), visible_gpus())
    cmd = launcher_command(n, argv, free_port(), script)
    print("[bench] launching: " + " ".join(cmd), file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    line = None
    for ln in proc.stdout:
        if ln.startswith("{") and '"metric"' in ln:
            line = ln.strip()
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = proc.wait()
    if rc != 0:
        print(f"[bench] a rank failed (exit {rc})", file=sys.stderr, flush=True)
        return rc
    if line is None:
        print("[bench] rank 0 printed no result line", file=sys.stderr, flush=True)
        return 1
    print(line, flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--nll-images", type=int, default=10000)
    ap.add_argument("--nll-k", type=int, default=5000)
    ap.add_argument("--no-nll", action="store_true")
    ap.add_argument("--no-large-batch", action="store_true")
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--large-batch-steps", type=int, default=20)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-c0", action="store_true")
    ap.add_argument("--c0-steps", type=int, default=200)
    ap.add_argument("--tune", action="append", default=[],
                    help="library tuning knob name=value (include/iwae.h enum iwae_knob), repeatable; A/B runs only")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    backend = dist_backend()
    if world != args.gpus:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; reporting the {world} ranks that run",
              file=sys.stderr, flush=True)
    ngpu = visible_gpus()
    if world > 1:
        check_world(world, backend, ngpu)
    # one process per GPU; only the gloo rehearsal shares a GPU between ranks
    dev = local if backend == "nccl" or world == 1 else local % max(1, ngpu)
    if dev >= ngpu:
        raise SystemExit(f"LOCAL_RANK {local} has no GPU ({ngpu} visible)")
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    from iwae_replication_project_amd import Adam, Flexible_Model, distributed

    x_all, pi = synthetic_images(50_000, 1 + rank)
    tuning = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in args.tune}
    model = Flexible_Model(HE, HD, LE, LD, dataset_bias=pi, loss_function="IWAE", k=K, seed=2,
                           use_graphs=not args.no_graphs, tuning=tuning)
    model.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
    if world > 1:
        distributed.enable_data_parallel(model)
    import ctypes
    dpw, dpc = ctypes.c_int(0), ctypes.c_int(0)
    model._call(model._lib.iwae_dp_world(model._h, ctypes.byref(dpw), ctypes.byref(dpc)))
    rccl_world = dict(torch_world=dist.get_world_size() if world > 1 else 1, backend=backend if world > 1 else None,
                      library_dp_world=dpw.value, library_rccl_comm_ranks=dpc.value,
                      train_reduce=(model._dp.comm if model._dp is not None else None))
    if world > 1 and backend == "nccl" and (dpc.value != world or dpw.value != world):
        # the N > 1 headline must run the library's in-graph RCCL all-reduce over every rank
        raise SystemExit(f"[bench] rank {rank}: library RCCL communicator has {dpc.value} ranks, data-parallel "
                         f"world {dpw.value}; expected {world}")
    xd = model._x(x_all)
    nb = xd.shape[0] // B_PER_GPU
    batches = [xd[i * B_PER_GPU:(i + 1) * B_PER_GPU] for i in range(nb)]

    def barrier():
        if world > 1:
            dist.barrier()

    def run(n, off=0):
        # fit's batch loop (E:82): consecutive batches of the resident set, one
        # library call per contiguous run (iwae_train_steps: up to 32 steps per graph)
        while n > 0:
            o = off % nb
            m = min(n, nb - o)
            model.train_steps(xd[o * B_PER_GPU:(o + m) * B_PER_GPU], B_PER_GPU, sync=False)
            n -= m
            off += m

    def run_calls(n, off=0):
        # the same steps as one train_step call each (F:221 per call)
        for i in range(n):
            model.train_step(batches[(off + i) % nb], sync=False)

    def prepare(n, off=0):
        # capture (without running) every graph run(n, off) replays: the timed
        # region then measures fit's steady-state loop, not graph capture
        while n > 0:
            o = off % nb
            m = min(n, nb - o)
            model.prepare_train_steps(xd[o * B_PER_GPU:(o + m) * B_PER_GPU], B_PER_GPU)
            n -= m
            off += m

    # ---- the timed call's graphs captured and uploaded (no step runs), then the
    # W warmup steps, so the timed call starts on a GPU that has just been busy
    # (not one left idle while the host captured and instantiated its graphs)
    prepare(args.steps, args.warmup)
    run(args.warmup)
    model._stream.synchronize()
    torch.cuda.synchronize()
    cap0 = model.graph_captures()
    # ---- timed region: K train steps
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps, args.warmup)
    model._stream.synchronize()
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    captures_timed = model.graph_captures() - cap0
    if captures_timed:
        raise SystemExit(f"[bench] {captures_timed} graph capture(s) inside the timed region")
    # no in-launch wait of the timed steps gave up (their gradients would be invalid)
    model.check_kernel_status()
    if world > 1:
        t = torch.tensor([el], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    rows = world * B_PER_GPU * K * args.steps
    value = rows / el
    ms_per_step = 1e3 * el / args.steps
    # the same number of steps as one train_step call each (host issue + one graph per step)
    run_calls(min(args.warmup, 10), args.warmup + args.steps)
    model._stream.synchronize()
    barrier()
    torch.cuda.synchronize()
    tc0 = time.perf_counter()
    run_calls(args.steps, 2 * args.warmup + args.steps)
    model._stream.synchronize()
    torch.cuda.synchronize()
    barrier()
    elc = time.perf_counter() - tc0
    if world > 1:
        t = torch.tensor([elc], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elc = float(t.item())
    loss = float(model._loss_buf.item())
    per_call = dict(ms_per_step=round(1e3 * elc / args.steps, 5), value=round(rows / elc, 1),
                    note="the same steps issued as one train_step (F:221) call each: one graph launch per step")

    # ---- dominant kernel live timing.  Candidates: the train engine's forward and
    # backward launches (iwae_train.hip) and, where the step still uses it, the
    # output-layer Bernoulli GEMM.  Each is recorded from one eager step and
    # re-launched K times back to back between two HIP events on the library's
    # stream (the stream it runs on); avg = elapsed / K.  The dominant one (the
    # longest) is priced against its matrix-core peak.

    def live(kind, epi):
        model._call(model._lib.iwae_profile_gemm(model._h, kind, epi))
        run(1, args.warmup + args.steps)
        ms, fl = ctypes.c_double(), ctypes.c_double()
        rc = model._lib.iwae_profile_replay(model._h, args.steps, ctypes.byref(ms), ctypes.byref(fl))
        model._call(model._lib.iwae_profile_gemm(model._h, -1, -1))
        if rc != 0:
            return None
        return ms.value / args.steps, fl.value / args.steps

    # algorithmic FLOP and bytes per launch (kernel_work): the forward and backward
    # launches each do one product per sample-row Dense layer (281,800 MACs per
    # row); the library's own count of the forward includes the
    # output MLP's two hidden layers that its column-split jobs recompute
    # (reported as executed).  Each kernel is priced against the roofline its
    # FLOP / byte ratio puts it under (roofline_of).
    rows_step = B_PER_GPU * K
    specs = {"tc_kernel forward (train engine, bf16x3)": (10, 0, "fwd"),
             "tc_kernel backward (train engine, bf16x3)": (11, 0, "bwd"),
             "upd_kernel (weight gradients + Adam + FX copies, bf16x3)": (15, 0, "upd"),
             "tcu_kernel (job I' + weight gradients + Adam + FX copies, one launch)": (16, 0, "tcu")}
    kern = {}
    for name, (kind, epi, wk) in specs.items():
        v = live(kind, epi)
        if v is None:
            continue
        fl, nby = kernel_work(wk, rows_step, B_PER_GPU)
        r = roofline_of(fl, nby, v[0] * 1e3)
        kern[name] = dict(avg_us=round(v[0] * 1e3, 3), flop_per_launch=fl, flop_executed=v[1],
                          alg_bytes_per_launch=nby, tflops=round(fl / (v[0] * 1e-3) / 1e12, 3),
                          bound=r["bound"], frac=r["frac"], flop_per_byte=r["flop_per_byte"])
    dom = max(kern, key=lambda k: kern[k]["avg_us"])
    kd = kern[dom]
    # HBM traffic of the same kernel: committed rocprofv3 PMC record (tools/pmc_passes.sh +
    # tools/pmc_to_json.py; FETCH_SIZE x2 per the gfx950 correction, WRITE_SIZE as is)
    traffic, traffic_src = None, None
    pmc_name = PMC_RECORD
    pmc = os.path.join(ROOT, "profiles", pmc_name)
    if os.path.exists(pmc):
        with open(pmc) as f:
            rec = json.load(f).get(dom)          # records keyed by the kernel label used here
        if rec:
            traffic = round(rec["traffic_bytes"] / 1e6, 3)
            traffic_src = f"profiles/{pmc_name} (MB per launch: fetch {rec['fetch_bytes'] / 1e6:.2f} + " \
                          f"write {rec['write_bytes'] / 1e6:.2f})"
    fl, nby = kd["flop_per_launch"], kd["alg_bytes_per_launch"]
    roofline = roofline_of(fl, nby, kd["avg_us"])
    roofline.update(traffic=traffic, traffic_unit="MB/launch", traffic_source=traffic_src,
                    traffic_over_alg=(round(traffic * 1e6 / nby, 2) if traffic else None),
                    kernel=dom, avg_us=kd["avg_us"], flop_per_launch=fl, alg_MB_per_launch=round(nby / 1e6, 3),
                    launches=args.steps,
                    peak_basis=("mfma: bf16 dense 2.5 PFLOP/s / 3 bf16 MFMAs per bf16x3 product; hbm: 8 TB/s; "
                                "bound = the larger of FLOP / 833.3 TFLOP/s and bytes / 8 TB/s (ridge 104 FLOP/B)"),
                    mfma_frac=round(fl / (kd["avg_us"] * 1e-6) / 1e12 / BF16X3_PEAK_TFLOPS, 4),
                    frac_of_bf16_dense_peak=round(fl / (kd["avg_us"] * 1e-6) / 1e12 / BF16_PEAK_TFLOPS, 4),
                    kernels=kern, step_tflops=round(TRAIN_FLOP_PER_ROW * rows / el / 1e12, 3))

    # ---- the train step's memory-bound launches (Adam, bound, FX refresh), same
    # replay timing: algorithmic HBM bytes per launch / duration vs HBM peak
    mem = {}
    for kind, name in ((12, "adam_kernel"), (13, "bound_kernel"), (14, "fx_refresh_kernel")):
        v = live(kind, 0)
        if v is not None:
            ms1, by = v
            mem[name] = dict(avg_us=round(ms1 * 1e3, 3), bytes_per_launch=int(by),
                             gbps=round(by / (ms1 * 1e-3) / 1e9, 1),
                             frac_of_hbm_peak=round(by / (ms1 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
    roofline["memory_kernels"] = dict(peak_gbps=HBM_PEAK_GBS, kernels=mem,
                                      note="bytes: algorithmic (each operand once); launches replayed back to back")

    # ---- configs[4] per-GPU share: B=512 images per GPU, k=50, same model and
    # step (RCCL gradient all-reduce for N > 1)
    large = None
    if not args.no_large_batch:
        bl = LARGE_B_PER_GPU
        xl = model._x(synthetic_images(4 * bl, 7 + rank)[0])
        # fit's batch loop (E:82) as the headline leg times it: the steps' batches
        # (four distinct ones, repeated) contiguous, one train_steps call
        nls = args.large_batch_steps
        xls = xl.repeat((nls + 3) // 4, 1)[:nls * bl].contiguous()
        model.train_steps(xls, bl, sync=False)           # warm-up: captures the multi-step graph
        model._stream.synchronize()
        cap1 = model.graph_captures()
        barrier()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        model.train_steps(xls, bl, sync=False)
        model._stream.synchronize()
        torch.cuda.synchronize()
        barrier()
        el3 = time.perf_counter() - t2
        if model.graph_captures() != cap1:
            raise SystemExit("[bench] graph capture inside the large-batch timed region")
        model.check_kernel_status()
        if world > 1:
            t = torch.tensor([el3], device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el3 = float(t.item())
        lrows = world * bl * K * args.large_batch_steps
        ltf = TRAIN_FLOP_PER_ROW * lrows / el3 / 1e12
        large = dict(value=round(lrows / el3, 1), unit="image*samples/s", per_gpu_batch=bl, global_batch=bl * world,
                     k=K, steps=args.large_batch_steps, ms_per_step=round(1e3 * el3 / args.large_batch_steps, 4),
                     tflops=round(ltf, 3), frac_of_peak=round(ltf / (BF16X3_PEAK_TFLOPS * world), 4),
                     peak_basis="bf16x3 products: bf16 dense 2.5 PFLOP/s / 3 = 833.3 TFLOP/s per GPU",
                     workload="BASELINE configs[4] per-GPU share (4096 over 8 GPUs)",
                     loop="Flexible_Model.train_steps over the steps' batches (fit's loop, E:82)",
                     precision=PRECISION)
        # the step's kernels against their rooflines: committed rocprofv3 kernel trace + PMC
        # record of the same step (tools/gpu_lbpmc.sh -> tools/lb_record.py)
        lbr = os.path.join(ROOT, "profiles", LB_RECORD)
        if os.path.exists(lbr):
            with open(lbr) as f:
                kr = json.load(f)
            ks = kr.get("kernels", {})
            pr = {k: v for k, v in ks.items() if "frac" in v and "bound" in v}
            if pr:
                dom = max(pr, key=lambda k: pr[k]["avg_us"])
                d = pr[dom]
                large["roofline"] = dict(bound=d["bound"], kernel=dom, achieved=d.get("achieved"), peak=d.get("peak"),
                                         unit=d.get("unit"), frac=d["frac"], avg_us=d["avg_us"],
                                         flop_per_byte=d.get("flop_per_byte"),
                                         alg_MB_per_launch=d.get("alg_MB_per_launch"),
                                         traffic=d.get("hbm_MB_per_launch"), traffic_unit="MB/launch",
                                         source=f"profiles/{LB_RECORD} (rocprofv3 trace + PMC of "
                                                "tools/train_large.py 512; tools/lb_record.py)")
            large["kernels"] = ks

    # ---- k=5000 NLL over the test images, sharded by image
    nll = None
    if not args.no_nll:
        xt, _ = synthetic_images(args.nll_images, 99)
        lo, hi = distributed.shard_range(args.nll_images, rank, world)
        xs = model._x(xt[lo:hi])
        # warm the NLL workspace and the torch ops of the bookkeeping below (their first
        # use loads GPU code objects: tens to hundreds of ms, not NLL work)
        # (a full chunk of images: the workspace reaches its final size here, not in the timed call)
        lpw = model.log_px(xs[: max(1, min(hi - lo, (1 << 20) // args.nll_k))], args.nll_k)
        torch.stack([lpw.sum(), torch.tensor(1.0, device=lpw.device)])
        barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        lp = model.log_px(xs, args.nll_k)        # per-image log p(x); returns after its stream drained
        torch.cuda.synchronize()
        barrier()
        el2 = time.perf_counter() - t1
        tot = torch.stack([lp.sum(), torch.tensor(float(hi - lo), device=lp.device)])
        if world > 1:
            t = torch.tensor([el2], device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el2 = float(t.item())
            dist.all_reduce(tot)
        nll = dict(value=round(args.nll_images / el2, 2), unit="images/s", images=args.nll_images, k=args.nll_k,
                   seconds=round(el2, 4), nll=round(float(-(tot[0] / tot[1]).item()), 4), shard="image",
                   n_gpus=world, images_per_rank=[distributed.shard_range(args.nll_images, r, world)[1] -
                                                  distributed.shard_range(args.nll_images, r, world)[0]
                                                  for r in range(world)],
                   tflops=round(NLL_FLOP_PER_IMAGE * (args.nll_k / 5000) * args.nll_images / el2 / 1e12, 3),
                   precision="bf16x3")
        if world > 1:
            # the 1-GPU rate on this node: rank 0 alone over every image (the others wait),
            # so the sharded rate reads as a fraction of N x the 1-GPU rate
            barrier()
            single = None
            if rank == 0:
                xa = model._x(xt)
                torch.cuda.synchronize()
                t5 = time.perf_counter()
                model.log_px(xa, args.nll_k)
                torch.cuda.synchronize()
                single = args.nll_images / (time.perf_counter() - t5)
                del xa
            barrier()
            if rank == 0:
                nll.update(one_gpu_value=round(single, 2), frac_of_linear=round(nll["value"] / (world * single), 4),
                           one_gpu_note="rank 0 alone over all images, same run, after the sharded leg")

    # ---- get_training_statistics (F:496-F:526) over the 10k synthetic test images
    # at the model's k: VAE, IWAE, E_q log p(x|h), both KLs, reconstruction loss
    # (chunks of 2000 images), two k=5000 NLL passes over all images (F:515,
    # F:518), 1000 encoder draws for the unit activity (F:521), LL_pruned (F:524)
    stats = None
    if not args.no_stats and world == 1:
        xt, _ = synthetic_images(args.nll_images, 99)
        xs = model._x(xt)
        model.get_training_statistics(xs[:200], K, batch_size=10)     # warm the shapes' workspaces
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        res, res2 = model.get_training_statistics(xs, K, batch_size=10)
        torch.cuda.synchronize()
        el5 = time.perf_counter() - t4
        stats = dict(value=round(args.nll_images / el5, 1), unit="images/s", seconds=round(el5, 4),
                     images=args.nll_images, k=K, batch_size=10, nll=round(res["NLL"], 4),
                     active_units=res2["number_of_active_units"],
                     workload="get_training_statistics (F:496-F:526) over the synthetic test set, batched "
                              "(per-batch reductions kept; two k=5000 NLL passes over all images)")

    # ---- configs[0]: 1 stochastic layer 784-200-200-50, IWAE k=5, batch 20 per GPU
    c0 = None
    if not args.no_c0:
        m0 = Flexible_Model([200], [200], [50], [784], dataset_bias=pi, loss_function="IWAE", k=5, seed=2,
                            use_graphs=not args.no_graphs, tuning=tuning)
        m0.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
        if world > 1:
            distributed.enable_data_parallel(m0)
        for i in range(10):
            m0.train_step(batches[i % nb], sync=False)
        m0._stream.synchronize()
        barrier()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        for i in range(args.c0_steps):
            m0.train_step(batches[i % nb], sync=False)
        m0._stream.synchronize()
        torch.cuda.synchronize()
        barrier()
        el4 = time.perf_counter() - t3
        if world > 1:
            t = torch.tensor([el4], device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el4 = float(t.item())
        c0rows = world * B_PER_GPU * 5 * args.c0_steps
        c0 = dict(value=round(c0rows / el4, 1), unit="image*samples/s", workload="BASELINE configs[0]: IWAE k=5, "
                  "1 stochastic layer 784-200-200-50, batch 20 per GPU", steps=args.c0_steps,
                  ms_per_step=round(1e3 * el4 / args.c0_steps, 5),
                  tflops=round(1_438_240 * c0rows / el4 / 1e12, 3))

    cpu = cpu_nll = cpu_c0 = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.cpu_seconds)
        cpu_nll = cpu_baseline_nll(max(4.0, args.cpu_seconds / 2))
        if c0 is not None:
            cpu_c0 = cpu_baseline_configs0(max(2.0, args.cpu_seconds / 3))

    if rank == 0:
        out = {
            "metric": "train images*k/sec and k=5000 test-NLL images/sec, 1-8 MI355X",
            "value": round(value, 1),
            "unit": "image*samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32 (bf16x3 split products)",
            "precision": PRECISION,
            "data": "synthetic",
            "config": {"workload": "IWAE train step (fwd+bound+bwd+Adam), k=50, 2 stochastic layers "
                                   "784-200-200-100-100-50, batch 20 per GPU (BASELINE configs[1])",
                       "global_batch": B_PER_GPU * world, "k": K, "parallelism": f"dp{world}",
                       "noise": "device Philox", "graphs": not args.no_graphs,
                       "loop": "fit's batch loop (E:82): consecutive batches through Flexible_Model.train_steps "
                               "(iwae_train_steps, up to 32 captured steps per graph launch); the timed call's "
                               "graphs are captured before the clock starts (iwae_train_steps_prepare)",
                       "graph_captures_in_timed_region": captures_timed},
            "loss": round(loss, 4),
            "train_step_calls": per_call,
            "rccl_world": rccl_world,
            "nll": nll,
            "large_batch": large,
            "training_statistics": stats,
            "configs0_train": c0,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "cpu_baseline_nll": cpu_nll,
            "cpu_baseline_configs0": cpu_c0,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
