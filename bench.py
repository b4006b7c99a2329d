"""Benchmark: EBSD VAE training step on MI355X (BASELINE.json config c2/c3).

One "step" = forward (encoder -> reparameterise -> decoder) + BCE/KL loss + backward +
(N>1: RCCL gradient all-reduce) + Adam, on B synthetic 128x128 fp32 patterns per GPU
(weak scaling), seeded kaiming-uniform weights of the reference architecture.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 256]
    torchrun --nproc-per-node N ... bench.py --gpus N ...     (N > 1, one rank per GPU)

Prints ONE JSON line (rank 0) with the driver's contract fields plus:
  roofline      the dominant kernel family (by GPU time), its algorithmic FLOPs per
                launch / average launch duration (HIP events on the launch stream, live in
                the timed region on every --probe-every'th step) against the peak of the
                conv arithmetic (fp16/bf16 MFMA / products per fp32 product, or fp32 MFMA);
                roofline.step: the attainable-roofline fraction of the whole step,
                sum_k max(F_k / P_k, B_k / BW) / T;
  strict_fp32   the same step with every conv on v_mfma_f32 (no split arithmetic);
  c5_256        the c5 configuration (256x256, latent 64, batch 128/GPU) step rate;
  c4_encoder_latents  build_dictionary throughput through the unmodified
                DiffractionPatternIndexer loop (one model(x) call per batch, mu kept) and a
                batched query;
  cpu_baseline  oracle/torch_port.py (PyTorch-CPU restatement of the reference
                training_step) on this host's cores, at BASELINE.md section 4's shapes
                (B=8, B=256, encoder-only B=1024; N=1, rank 0).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

# Hardware queues per process (read once, when the HIP runtime initialises): an RCCL process
# group's streams take HW queues of their own, and at HIP's default of 4 the weight-gradient
# side stream then shares a queue with the main stream -- measured on one GPU with a world-1
# `nccl` group: 9.30 ms per step at 4 queues, 8.55 at 8 (tools/bucket_ab.py)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "ebsd-vae_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_PEAK_TFLOPS = 157.3      # MI355X fp32 MFMA (= fp32 vector) dense peak
HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def step_flops_per_pattern(plan) -> float:
    """Algorithmic FLOPs of one pattern through fwd + bwd (convs + linears)."""
    from latice.engine import conv_flops
    f = 0.0
    for i, L in enumerate(plan.enc + plan.dec):
        c = conv_flops(1, L.H, L.H, L.cin, L.cout)
        f += c * (2 if (i == 0) else 3)          # fwd + wgrad (+ dgrad except the first conv)
    S = plan.image_size
    f += 3 * conv_flops(1, S, S, plan.inplanes, 1)  # final conv fwd + dgrad + wgrad
    lin = 2 * plan.feat * plan.latent_dim * 3       # mu, logvar, linear2
    return f + 3 * lin


PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def pmc_traffic(fam: str):
    """HBM bytes per launch of `fam` from the committed rocprofv3 PMC passes
    (tools/pmc_traffic.py: (2*FETCH_SIZE + WRITE_SIZE) KiB, gfx950 fetch correction)."""
    try:
        with open(PMC_SUMMARY) as f:
            t = json.load(f)["traffic"][fam]
        return t["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def _cpu_name():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(plan, timed: int = 3):
    """the PyTorch-CPU restatement of the reference training step
    (oracle/torch_port.py, parity-pinned to the reference's golden vectors) on all of this
    rank's host cores: B=8 (c1), B=256 (c2's shape) fwd+loss+bwd+Adam and encoder+mu at
    B=1024 (c4), each 1 warm-up + the median of `timed` steps.  value = the B=256 rate."""
    from latice.seeding import seeded_state_dict, synthetic_patterns
    from oracle.torch_port import CPUStep   # oracle: the baseline leg only
    # the box's CPU share: OMP_NUM_THREADS when set (the affinity mask can list every CPU of
    # the machine while the job's quota is far smaller: oversubscribing it is 10x slower)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    torch.set_num_threads(threads)
    sd = seeded_state_dict(0, plan.inplanes, plan.latent_dim, plan.image_size)
    S, L = plan.image_size, plan.latent_dim

    def median_rate(fn, batch):
        log(f"[bench] cpu baseline: batch {batch} on {threads} threads")
        x = torch.from_numpy(synthetic_patterns(123, batch, S))
        eps = torch.randn(batch, L)
        fn(x[: min(batch, 8)], eps[: min(batch, 8)])     # warm-up (allocator, oneDNN)
        ts = []
        for _ in range(timed):
            t0 = time.perf_counter()
            fn(x, eps)
            ts.append(time.perf_counter() - t0)
            log(f"[bench]   {ts[-1]:.2f} s")
        return batch / float(np.median(ts)), float(np.median(ts))

    st = CPUStep(sd, kl_lambda=5e-6)
    r8, t8 = median_rate(st.step, 8)
    r256, t256 = median_rate(st.step, 256)
    renc, tenc = median_rate(lambda x, e: st.encode(x), 1024)
    return {"value": round(r256, 3), "unit": "patterns/s", "cores": threads, "kind": "port",
            "sample": f"median of {timed} timed steps (after a warm-up) of fwd+loss+bwd+Adam at batch "
                      f"256, {S}x{S}, PyTorch-CPU restatement of the reference training_step "
                      f"(oracle/torch_port.py), {threads} threads, {_cpu_name()}",
            "b8_patterns_per_s": round(r8, 3), "b8_s_per_step": round(t8, 4),
            "b256_s_per_step": round(t256, 3),
            "encoder_b1024_latents_per_s": round(renc, 2), "encoder_b1024_s_per_batch": round(tenc, 3)}


class _SyntheticPatternLoader:
    """A DPDataModule test_dataloader stand-in over synthetic raw patterns: each batch is the
    on-device DPdataset transform (ebsdvae_ingest_patterns) of a raw float64 batch, with its
    angles -- what build_dictionary's loop consumes.  raw on the device: the batch is already
    resident in HBM.  raw in pinned host memory (h2d): every batch is first copied host ->
    device (the reference's `data.to(device)`, latice/index/dp_indexer.py:281, here of the raw
    float64 batch) on a copy stream, double-buffered so batch i+1's copy runs under batch i's
    encode."""

    def __init__(self, raw, image_size, nb, angles, device=None):
        from latice.data_module import ingest_patterns
        self._ingest = ingest_patterns
        self.raw, self.S, self.nb, self.angles = raw, image_size, nb, angles
        dev = raw.device if device is None else device
        self.x = torch.empty(raw.shape[0], 1, image_size, image_size, dtype=torch.float32,
                             device=dev)
        self.h2d = raw.device.type == "cpu"
        if self.h2d:
            self.bufs = [torch.empty(raw.shape, dtype=raw.dtype, device=dev) for _ in range(2)]
            self.copy = torch.cuda.Stream(device=dev)

    def __len__(self):
        return self.nb

    def __iter__(self):
        B = self.raw.shape[0]
        if not self.h2d:
            for i in range(self.nb):
                yield (self._ingest(self.raw, (self.S, self.S), out=self.x),
                       torch.from_numpy(self.angles[i * B:(i + 1) * B]))
            return
        main = torch.cuda.current_stream(self.x.device)
        done = [None, None]

        def fetch(i):
            buf = self.bufs[i % 2]
            self.copy.wait_stream(main)   # the ingest that last read this buffer is done
            with torch.cuda.stream(self.copy):
                buf.copy_(self.raw, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.copy)
            done[i % 2] = ev

        fetch(0)
        for i in range(self.nb):
            main.wait_event(done[i % 2])
            x = self._ingest(self.bufs[i % 2], (self.S, self.S), out=self.x)
            if i + 1 < self.nb:
                fetch(i + 1)
            yield x, torch.from_numpy(self.angles[i * B:(i + 1) * B])


def encoder_latents(model, plan, args, dev, world):
    """BASELINE c4: DiffractionPatternIndexer.build_dictionary (latice/index/dp_indexer.py:
    92-111, 254-297) at batch 1024 per GPU through the UNMODIFIED loop of the drop-in
    indexer: per batch the on-device transform, ONE `self.model(data)` call whose `[2]` is
    kept (the model's eval/no-grad forward defers the decoder, so it runs encoder + heads),
    `mu.cpu().numpy()`; then `db.add_vectors` into the HBM dictionary.  c4_batches (default
    1024 = 1,048,576 patterns) are split over the ranks; no collective.  Then one batched
    query of 4096 latents: cosine top-20 + orientation consensus."""
    import contextlib
    import logging
    from latice import engine as E
    from latice.index.dp_indexer import DiffractionPatternIndexer, IndexerConfig
    from latice.index.faiss_db import FaissLatentVectorDatabase, FaissLatentVectorDatabaseConfig
    logging.getLogger("latice.index.faiss_db").setLevel(logging.ERROR)   # random angles never agree
    B, S = 1024, args.image_size
    H0 = S + 12   # raw patterns a little larger than the crop, as in the reference pipeline
    nb = max(1, args.c4_batches // world)
    gen = torch.Generator(device=dev).manual_seed(7 + dist.get_rank() if world > 1 else 7)
    raw = torch.rand(B, H0, H0, dtype=torch.float64, device=dev, generator=gen)
    angles = np.random.default_rng(11).uniform(0.0, 360.0, (nb * B, 3))
    db = FaissLatentVectorDatabase(FaissLatentVectorDatabaseConfig(
        npz_path="/nonexistent/c4_dictionary.npz", dimension=plan.latent_dim, device=str(dev)))
    db.reserve(nb * B)
    cfg = IndexerConfig(pattern_path="/nonexistent/patterns.npy", angles_path="/nonexistent/angles.txt",
                        batch_size=B, device="cuda", latent_dim=plan.latent_dim, image_size=(S, S))
    ix = DiffractionPatternIndexer(model, db=db, config=cfg)
    quiet = contextlib.redirect_stdout(sys.stderr)   # the indexer's progress bar
    with quiet:
        ix._extract_latent_vectors_with_angles(_SyntheticPatternLoader(raw, S, 2, angles))  # warm-up
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with quiet:
        lat, ori = ix._extract_latent_vectors_with_angles(_SyntheticPatternLoader(raw, S, nb, angles))
        ix.db.add_vectors(lat, ori)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    finite = bool(np.isfinite(lat).all())
    # the same loop with every raw float64 batch copied host -> device first (pinned memory,
    # copy stream, double-buffered): the PCIe-inclusive rate beside the HBM-resident one
    nh = min(nb, args.c4_h2d_batches)
    h2d = None
    if nh > 0:
        raw_h = raw.cpu().pin_memory()
        with quiet:
            ix._extract_latent_vectors_with_angles(_SyntheticPatternLoader(raw_h, S, 2, angles, dev))
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        th = time.perf_counter()
        with quiet:
            ix._extract_latent_vectors_with_angles(_SyntheticPatternLoader(raw_h, S, nh, angles, dev))
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        hel = time.perf_counter() - th
        if world > 1:
            t = torch.tensor([hel], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            hel = float(t)
        h2d = {"value": round(world * B * nh / hel, 1), "unit": "latents/s", "batches": nh,
               "ms_per_batch": round(hel / nh * 1e3, 3),
               "raw_batch_mb": round(raw_h.numel() * 8 / 1e6, 1),
               "what": "the same unmodified loop with each raw float64 batch copied from pinned host "
                       "memory to the GPU first (dp_indexer.py:281 data.to(device)); copy stream, "
                       "double-buffered under the previous batch's encode"}
        del raw_h
    # the encoder-only engine loop without the per-batch host copy, for comparison
    params = dict(model.named_parameters())
    packs = model._inference_packs(params)
    x = torch.empty(B, 1, S, S, dtype=torch.float32, device=dev)
    ne = min(nb, 64)
    with torch.no_grad():
        from latice.data_module import ingest_patterns
        E.encode_latents(plan, ingest_patterns(raw, (S, S), out=x), params, packs)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(ne):
            mu = E.encode_latents(plan, ingest_patterns(raw, (S, S), out=x), params, packs)
        torch.cuda.synchronize()
        eng = time.perf_counter() - t1
        # attainable time of one batch: the encoder's conv launches from one
        # event-bracketed encode (max(F/P, B/BW) each) + the transform's HBM bytes (read the
        # float64 raw batch, write the fp32 crop)
        with E.probe() as probe:
            E.encode_latents(plan, ingest_patterns(raw, (S, S), out=x), params, packs)
        torch.cuda.synchronize()
        conv_att = probe.attainable_s(HBM_PEAK_GBS * 1e9)
        ingest_att = (8.0 * B * H0 * H0 + 4.0 * B * S * S) / (HBM_PEAK_GBS * 1e9)
        heads_att = (4.0 * B * plan.feat + 4.0 * 2 * plan.feat * plan.latent_dim) / (HBM_PEAK_GBS * 1e9)
        # query leg: 4096 perturbed latents, top-20 + consensus over the whole dictionary
        q = (mu.repeat(4, 1) + 0.01 * torch.randn(4 * B, plan.latent_dim, device=dev, generator=gen))
        db.find_best_orientations_batch(q[:64], top_n=20)   # warm-up
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res = db.find_best_orientations_batch(q, top_n=20)
        torch.cuda.synchronize()
        qel = time.perf_counter() - t2
    if world > 1:
        t = torch.tensor([el, qel, eng], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, qel, eng = float(t[0]), float(t[1]), float(t[2])
    n = world * B * nb
    enc_flops = sum(2.0 * L.H * L.H * L.cin * L.cout * 9 for L in plan.enc) + 2 * plan.feat * plan.latent_dim
    return {"metric": "encoder latents/sec (c4: DiffractionPatternIndexer.build_dictionary loop = "
                      "on-device transform + model(x)[2] + mu.cpu() per batch + dictionary add, "
                      "batch 1024/GPU)",
            "value": round(n / el, 1), "unit": "latents/s", "latents": n,
            "ms_per_batch": round(el / nb * 1e3, 3),
            "tflops": round(enc_flops * n / el / 1e12, 2), "finite": finite,
            "roofline": {"definition": "sum_k max(F_k/P_k, B_k/BW) per batch / measured ms per batch "
                                       "(SURVEY.md 8d): encoder conv launches (event-probed) + "
                                       "transform + heads bytes",
                         "attainable_ms_per_batch": round((conv_att + ingest_att + heads_att) * 1e3, 3),
                         "conv_attainable_ms": round(conv_att * 1e3, 3),
                         "measured_ms_per_batch": round(el / nb * 1e3, 3),
                         "frac": round((conv_att + ingest_att + heads_att) / (el / nb), 4),
                         "engine_only_frac": round((conv_att + ingest_att + heads_att) / (eng / ne), 4)},
            "with_host_to_device_copy": h2d,
            "engine_only": {"value": round(world * B * ne / eng, 1), "unit": "latents/s",
                            "batches": ne, "what": "transform + encode_latents, no host copy"},
            "query": {"metric": "queries/sec (cosine top-20 over the dictionary + orientation "
                                "consensus, one batch per GPU)",
                      "value": round(world * len(res) / qel, 1), "unit": "queries/s",
                      "queries": world * len(res), "dictionary_rows_per_gpu": db.get_count(),
                      "ms": round(qel * 1e3, 3)}}


def c5_step_rate(args, dev, world, rank):
    """BASELINE c5: the same training step on 256x256 patterns, latent 64, batch 128 per GPU
    (per-GPU 128, global 128*N), weak scaling like the headline line;
    barrier + synchronize around the timed steps, max over ranks."""
    from latice.model import VariationalAutoEncoderRawData
    from latice.seeding import seeded_state_dict, synthetic_patterns
    from latice.trainer import VAETrainer
    S, L, B = 256, 64, 128
    model = VariationalAutoEncoderRawData(32, L, S)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in seeded_state_dict(5, 32, L, S).items()})
    model = model.to(dev)
    trainer = VAETrainer(model, kl_lambda=5e-6, lr=1e-4, seed=2000 + rank)
    x = torch.from_numpy(synthetic_patterns(100 + rank, B, S)).to(dev)
    for _ in range(3):
        trainer.step(x)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.c5_steps):
        out = trainer.step(x)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    loss = float(out[0])
    ms = el / args.c5_steps * 1e3
    step_tflops = step_flops_per_pattern(model.plan) * B * args.c5_steps / el / 1e12
    # the attainable step from one extra event-bracketed step after the timed
    # ones (serial streams, so every launch is timed alone), against the timed step time
    from latice import engine as E
    with E.probe() as probe, E.serial_streams():
        trainer.step(x)
    torch.cuda.synchronize()
    roof = step_roofline(probe, model.plan, B, ms, 1, trainer.numel)
    del trainer, model, x
    torch.cuda.empty_cache()
    return {"metric": "EBSD patterns/sec (256x256, latent 64, fwd+bwd)",
            "value": round(world * B * args.c5_steps / el, 2), "unit": "patterns/s",
            "batch_per_gpu": B, "global_batch": world * B, "steps": args.c5_steps,
            "ms_per_step": round(ms, 3),
            "roofline": {"step": roof},
            "step_fp32_tflops": round(step_tflops, 2), "loss_finite": bool(np.isfinite(loss))}


def step_roofline(probe, plan, B, ms, probed, nparams):
    """T_roof = sum_k max(F_k / P_k, B_k / BW) over the kernels of one
    step, divided by the measured step time.  Conv launches (fwd, input gradient, weight
    gradient) come from the probe with their algorithmic FLOPs, the peak of the arithmetic
    they ran in and their algorithmic I/O bytes; the HBM-bound rest of the fused step is
    counted by its algorithmic bytes: the final conv(32->1) forward and its fused backward
    (read the 32-channel input twice + logits / logit gradient), the first block's fused
    backward (read x), BCE+KL (read x_hat, x; write the logit gradient) and Adam (7 fp32
    streams over the flat parameters).  Also given against the strict fp32 peak (every
    conv at 157.3 TFLOP/s), the reading SURVEY.md section 8d states."""
    from latice.engine import conv_flops
    S = plan.image_size
    bw = HBM_PEAK_GBS * 1e9
    conv_s = probe.attainable_s(bw) / probed
    conv_fp32_s = sum(max(f / (FP32_PEAK_TFLOPS * 1e12), nb / bw)
                      for _, f, _, _, _, _, nb in probe.records) / probed
    px = B * S * S
    fin_f = conv_flops(B, S, S, plan.inplanes, 1)
    rest = [(fin_f, 4.0 * px * (plan.inplanes + 1)),            # final conv forward
            (2 * fin_f, 4.0 * px * (2 * plan.inplanes + 1)),     # its fused backward
            (0.0, 4.0 * px),                                      # first block: read x
            (0.0, 3 * 4.0 * px),                                  # BCE + KL fwd/bwd
            (0.0, 28.0 * nparams)]                                # Adam
    rest_s = sum(max(f / (FP32_PEAK_TFLOPS * 1e12), b / bw) for f, b in rest)
    t = ms / 1e3
    return {"definition": "sum_k max(F_k/P_k, B_k/BW) / T_step (SURVEY.md 8d)",
            "attainable_ms": round((conv_s + rest_s) * 1e3, 3), "measured_ms": round(ms, 3),
            "frac": round((conv_s + rest_s) / t, 4),
            "frac_vs_fp32_peak": round((conv_fp32_s + rest_s) / t, 4),
            "conv_attainable_ms": round(conv_s * 1e3, 3), "other_attainable_ms": round(rest_s * 1e3, 3)}


def strict_fp32_rate(model, x, args, dev, world):
    """The same training step with every conv on v_mfma_f32_32x32x2_f32 (no split
    arithmetic), timed like the headline line (barrier + synchronize, max over ranks)."""
    from latice import engine as E
    from latice.trainer import VAETrainer
    with E.precision("fp32"):
        tr = VAETrainer(model, kl_lambda=5e-6, lr=1e-4, seed=3000)
        for _ in range(2):
            tr.step(x)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.strict_fp32_steps):
            tr.step(x)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    del tr
    return {"value": round(world * x.shape[0] * args.strict_fp32_steps / el, 2), "unit": "patterns/s",
            "ms_per_step": round(el / args.strict_fp32_steps * 1e3, 3), "steps": args.strict_fp32_steps,
            "dtype": "fp32"}


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """`--gpus N` without a launcher: start N fresh child processes of this script, one per
    GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in their environment, as
    torch.distributed.run sets them), wait for all of them and return the worst exit code.
    The parent never touches HIP (torch.cuda.device_count() does not initialise it), so the
    children start on an untouched device; rank 0's JSON line goes to the shared stdout."""
    import signal
    import subprocess
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and ndev and args.gpus > ndev:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but only {ndev} visible GPU(s)")
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), EBSDVAE_BENCH_LAUNCHER="bench.py --gpus")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    for q in pending:          # a failed rank would leave the others waiting
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="patterns per GPU")
    ap.add_argument("--image-size", type=int, default=128)
    ap.add_argument("--latent-dim", type=int, default=16)
    ap.add_argument("--cpu-timed", type=int, default=3, help="timed CPU-baseline steps per shape")
    ap.add_argument("--strict-fp32-steps", type=int, default=20,
                    help="timed steps of the strict fp32-MFMA leg (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true", help="time without per-kernel events")
    ap.add_argument("--probe-every", type=int, default=10,
                    help="bracket the conv launches with HIP events on every k-th timed step")
    ap.add_argument("--precision", default=None, choices=["fp32", "bf16x6", "bf16x3", "f16x3"],
                    help="conv arithmetic (default: the engine default, f16x3)")
    ap.add_argument("--c4-batches", type=int, default=1024,
                    help="encoder-only inference batches of 1024 for the c4 latents/s field (0: skip)")
    ap.add_argument("--c4-h2d-batches", type=int, default=64,
                    help="batches of the c4 variant with the host->device copy of each raw batch (0: skip)")
    ap.add_argument("--c5-steps", type=int, default=10,
                    help="timed steps of the c5 leg (256x256, latent 64, batch 128/GPU; 0: skip)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="torch.distributed backend for N>1 (nccl = RCCL; gloo only to rehearse "
                         "several ranks on one GPU)")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="seconds before a stuck process-group init or collective raises")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:       # no launcher: spawn one rank per GPU, before any HIP call
            sys.exit(launch_ranks(args))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started "
                         f"WORLD_SIZE={os.environ['WORLD_SIZE']} ranks")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; modulo only matters when rehearsing several ranks on one GPU
    local = local % max(1, torch.cuda.device_count())
    pg = None
    if world > 1:
        import datetime
        torch.cuda.set_device(local)
        timeout = datetime.timedelta(seconds=args.dist_timeout)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"), timeout=timeout)
        else:
            dist.init_process_group(args.dist_backend, timeout=timeout)
        # what actually formed: the backend and the ranks of the group
        pg = {"backend": str(dist.get_backend()), "world_size": dist.get_world_size(),
              "launcher": os.environ.get("EBSDVAE_BENCH_LAUNCHER", "torch.distributed.run"),
              "devices": min(world, max(1, torch.cuda.device_count())),
              "timeout_s": args.dist_timeout}
        if pg["world_size"] != world:
            raise SystemExit(f"bench.py: process group has {pg['world_size']} ranks, expected {world}")
    dev = torch.device(f"cuda:{local}")

    from latice import engine as E
    from latice.model import VariationalAutoEncoderRawData
    if args.precision:
        E.set_precision(args.precision)
    from latice.seeding import seeded_state_dict, synthetic_patterns
    from latice.trainer import VAETrainer

    model = VariationalAutoEncoderRawData(32, args.latent_dim, args.image_size)
    sd = seeded_state_dict(0, 32, args.latent_dim, args.image_size)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model = model.to(dev)
    trainer = VAETrainer(model, kl_lambda=5e-6, lr=1e-4, seed=1000 + rank)
    x = torch.from_numpy(synthetic_patterns(rank, args.batch, args.image_size)).to(dev)
    plan = model.plan

    log(f"[bench] rank {rank}/{world} batch {args.batch} warmup {args.warmup} steps {args.steps}")
    # EBSDVAE_CU_SPLIT=k (experiment): the step runs on the N - k CU stream,
    # the weight gradients on the other k
    split_main = E.cu_split_main(dev)
    step_ctx = torch.cuda.stream(split_main) if split_main is not None else contextlib.nullcontext()
    step_ctx.__enter__()
    for _ in range(args.warmup):
        trainer.step(x)
    torch.cuda.synchronize()

    probe = E.probe() if not args.no_probe else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    probed = 0
    trainer.time_allreduce = world > 1   # one event pair per step around the exposed all-reduce
    for i in range(args.steps):
        if probe is not None and i % args.probe_every == 0:
            # event-bracketed launches on a sample of the timed steps: each event pair costs
            # the stream a few microseconds, so bracketing every launch of every step would
            # slow the step the value is quoted on by ~2 %.  These steps keep the weight
            # gradients on the main stream, so that every launch is timed alone (overlapped
            # launches would each carry the other's time); ~5 % slower, one step in ten
            with probe, E.serial_streams():
                out = trainer.step(x)
            probed += 1
        else:
            out = trainer.step(x)
    torch.cuda.synchronize()
    trainer.time_allreduce = False
    step_ctx.__exit__(None, None, None)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rank_ms = None
    if world > 1:
        # every rank's own time (the spread shows stragglers / RCCL waits), then the max
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        tg = t if dist.get_backend() == "nccl" else t.cpu()
        per = [torch.zeros_like(tg) for _ in range(world)]
        dist.all_gather(per, tg)
        rank_ms = [round(float(p) / args.steps * 1e3, 3) for p in per]
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    loss = float(out[0])
    ms = elapsed / args.steps * 1e3
    value = world * args.batch * args.steps / elapsed
    exposed = trainer.allreduce_exposed_ms()
    if exposed is not None:
        t = torch.tensor([exposed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        exposed = round(float(t), 4)

    roof = None
    fam = {}
    if probe is not None:
        fam = probe.summary()
        dom = max(fam, key=lambda k: fam[k]["ms"])
        d = fam[dom]
        flops_per_launch = d["flops"] / d["launches"]
        avg_s = d["ms"] / d["launches"] / 1e3
        ach = flops_per_launch / avg_s / 1e12
        # peak of the family's arithmetic (fp32 MFMA 157.3, or the bf16 MFMA peak over the
        # split's products per fp32 product), flop-weighted over its launches
        peak = d["flops"] / d["peak_s"] / 1e12
        roof = {"bound": "mfma", "kernel": dom, "achieved": round(ach, 2),
                "peak": round(peak, 1), "unit": "TFLOP/s",
                "frac": round(ach / peak, 4), "traffic": pmc_traffic(dom),
                "launches_per_step": d["launches"] // probed,
                "split_bf16_launches_per_step": d["split_launches"] // probed,
                "probed_steps": probed,
                "avg_launch_us": round(avg_s * 1e6, 2),
                "gflop_per_launch": round(flops_per_launch / 1e9, 3),
                "flops": "algorithmic fp32-equivalent (2*B*H*W*Cin*Cout*9 per conv)"}
        roof["step"] = step_roofline(probe, plan, args.batch, ms, probed, trainer.numel)
    step_tflops = step_flops_per_pattern(plan) * args.batch / (ms / 1e3) / 1e12

    prec = E.get_precision()
    first_conv = ("fp32 VALU (one fixed fma chain, ebsdvae_conv_first_fwd)" if E._first_valu(plan.enc[0])
                  else "fp32 MFMA (v_mfma_f32_32x32x2_f32)")
    res = {
        "metric": "EBSD patterns/sec (128x128, fwd+bwd)" if args.image_size == 128
        else f"EBSD patterns/sec ({args.image_size}x{args.image_size}, fwd+bwd)",
        "value": round(value, 2), "unit": "patterns/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": {"fp32": "fp32", "bf16x6": "fp32 I/O, bf16x6 split MFMA",
                  "bf16x3": "fp32 I/O, bf16x3 split MFMA",
                  "f16x3": "fp32 I/O, f16x3 split MFMA"}[prec],
        "data": "synthetic",
        "conv_arithmetic": prec + {
            "fp32": " (v_mfma_f32_32x32x2_f32; " + first_conv + " for the 1->32 conv)",
            "bf16x6": " (fp32 operands split into 3 bf16 pieces, 6 bf16 MFMA products per fp32"
                      " product, fp32 accumulation)",
            "bf16x3": " (2 bf16 pieces, 3 products: ~2^-16.5 per product)",
            "f16x3": " (fp32 operands split into 2 fp16 pieces, 3 fp16 MFMA products per fp32"
                     " product, ~2^-22.5, fp32 accumulation: forward, input-gradient and"
                     " weight-gradient convs; weights packed as w*2^k with one power of two per"
                     " layer from max|w|, the gradient operand scaled by a power of two per image"
                     " (input gradient) or per slice (weight gradient); " + first_conv +
                     " for the 1->32 conv, bf16x6 for the 8x8 weight gradient fed by an upsample; all"
                     " activations, statistics and reductions fp32/fp64; passes the fp32 parity"
                     " gates, tests/test_gpu_trainer.py)"}[prec],
        "config": {"workload": f"c{2 if world == 1 else 3}: VariationalAutoEncoderRawData "
                               f"{args.image_size}x{args.image_size}, latent {args.latent_dim}, "
                               f"batch {args.batch}/GPU, fwd+loss+bwd+Adam"
                               + (("" if pg is None else
                                   " + RCCL grad all-reduce" if pg["backend"] == "nccl" else
                                   f" + {pg['backend']} grad all-reduce (rehearsal, "
                                   f"{pg['devices']} GPU(s))")),
                   "global_batch": world * args.batch, "image_size": args.image_size,
                   "latent_dim": args.latent_dim, "parallelism": f"dp{world}"},
        "process_group": pg,
        "rank_ms_per_step": rank_ms,
        "allreduce_exposed_ms": exposed,
        "allreduce_exposed_what": ("GPU time per step (HIP events, max over ranks) from the end of the "
                                   "backward to the completion of the last gradient all-reduce: the "
                                   "exchange time no backward work hid (trainer.py)"
                                   if exposed is not None else None),
        "rank_spread_pct": (None if rank_ms is None else
                            round(100.0 * (max(rank_ms) - min(rank_ms)) / max(rank_ms), 2)),
        "roofline": roof,
        "step_fp32_tflops": round(step_tflops, 2),
        "step_frac_of_fp32_peak": round(step_tflops / FP32_PEAK_TFLOPS, 4),
        "loss": round(loss, 6),
        "kernel_families_ms_per_step": {k: round(v["ms"] / max(1, probed), 3) for k, v in fam.items()},
    }
    if args.strict_fp32_steps > 0:
        res["strict_fp32"] = strict_fp32_rate(model, x, args, dev, world)
    if args.c5_steps > 0 and args.image_size == 128:
        res["c5_256"] = c5_step_rate(args, dev, world, rank)
    if args.c4_batches > 0:
        res["c4_encoder_latents"] = encoder_latents(model, plan, args, dev, world)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("[bench] cpu baseline ...")
        res["cpu_baseline"] = cpu_baseline(plan, args.cpu_timed)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
