"""Training-throughput benchmark: BASELINE.json metric "training images/sec at 1280x720 bf16".

Workload (config.workload): one REFINE training step of the reference's train.py hot loop
(train.py:250-327) on synthetic BDD100K-shaped batches resident in HBM — normalise,
anchor matching, MobileNet-v2 + refine heads forward, smooth-L1 loss, backward, SGD+clip —
at 720x1280, batch 8 per GPU (configs[1] on one GPU; configs[2] = batch 64 on 8 GPUs is
the same per-GPU work, weak scaling).  Every kernel is librod (HIP, gfx950).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  N>1: launched by torch.distributed.run, one rank per GPU, RCCL all-reduce of the flat
  gradient buffer (sum, global-batch normalisation), clip after reduce.

Prints one JSON line (rank 0) with roofline (live HIP-event timing of the dominant
kernel over the timed region) and cpu_baseline (the oracle — a PyTorch-CPU restatement
of the same step — on a bounded sample, rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd')
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=8, help='images per GPU')
    ap.add_argument('--height', type=int, default=720)
    ap.add_argument('--width', type=int, default=1280)
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'fp32'])
    ap.add_argument('--train_range', default='REFINE', choices=['REFINE', 'ALL'])
    ap.add_argument('--augment', action='store_true', default=False,
                    help='each step starts from raw 720x1280 uint8 frames through the GPU training augmentation '
                         '(process_raw_data_train: random crop / resize / flip / colour, fused normalisation)')
    ap.add_argument('--no-fix-refine', dest='fix_refine', action='store_false', default=True,
                    help='ALL mode: train the backbone and refine heads too (train.py fix_refine=False)')
    ap.add_argument('--graph', dest='graph', action='store_true', default=True,
                    help='replay the training step as a HIP graph (Trainer.step_graphed; bit-identical to the '
                         'eager step).  N>1 over RCCL: the whole step, its bucketed all-reduces (on a side stream, '
                         'overlapping backward) included, through the library\'s communicator (\'full\')')
    ap.add_argument('--no-graph', dest='graph', action='store_false')
    ap.add_argument('--dp-leg', dest='dp_leg', action='store_true', default=True,
                    help='N=1: time the graphed step with a 1-rank RCCL reducer (the N>1 default: native, full '
                         'capture; with SyncBatchNorm; the torch.distributed split form) against the step without a '
                         'reducer ("dp_overhead")')
    ap.add_argument('--no-dp-leg', dest='dp_leg', action='store_false')
    ap.add_argument('--sync-bn', dest='sync_bn', action='store_true', default=False,
                    help='N>1: BatchNorm statistics over the global batch (rod.ddp.SyncBatchNorm; default per rank)')
    ap.add_argument('--probe', default='rod_dw3x3_bwd_fused,rod_dw3x3_bwd_fused_pw,rod_dw3x3_bwd_fused_rc',
                    help='C-ABI entry (or comma list, aggregated as one kernel family) reported in "roofline": '
                         'default the fused depthwise backward, the largest entry of the graphed step '
                         '(profiles/r3_refine_bf16_b8_720p_graph_stats.txt); rounds 1-2 reported the '
                         'BatchNorm backward (rod_bn_bwd_reduce,rod_bn_bwd_apply,rod_bn_bwd)')
    ap.add_argument('--probe-table', dest='probe_table', default=None,
                    help='time EVERY librod call and write a per-entry table (JSON) here (analysis only)')
    ap.add_argument('--traffic', default=os.path.join(ROOT, 'profiles', 'pmc_traffic.json'),
                    help='per-entry HBM bytes per launch from rocprofv3 PMC passes (tools/pmc_traffic.py)')
    ap.add_argument('--cpu-baseline', dest='cpu_baseline', action='store_true', default=True)
    ap.add_argument('--no-cpu-baseline', dest='cpu_baseline', action='store_false')
    ap.add_argument('--kernel-steps', dest='kernel_steps', type=int, default=2,
                    help='extra steps AFTER the timed region with the north-star kernels probed '
                         '("kernels" in the JSON: dw3x3 / pw GEMM / BN-backward rooflines); 0 = off')
    ap.add_argument('--inference', dest='inference', action='store_true', default=True)
    ap.add_argument('--no-inference', dest='inference', action='store_false')
    ap.add_argument('--inference-1080', dest='inference_1080', action='store_true', default=True)
    ap.add_argument('--no-inference-1080', dest='inference_1080', action='store_false')
    ap.add_argument('--fp32-leg', dest='fp32_leg', action='store_true', default=True,
                    help='N=1, bf16 run: also time the same step in fp32 (BASELINE configs[1] as stated, C2) '
                         'and report it under "training_fp32"')
    ap.add_argument('--no-fp32-leg', dest='fp32_leg', action='store_false')
    ap.add_argument('--tfrecord-leg', dest='tfrecord_leg', action='store_true', default=True,
                    help='N=1: feed the step from a TFRecord of synthetic 1280x720 JPEG frames through the '
                         'host JPEG decode + GPU augmentation (train.py input path) and report it under "tfrecord"')
    ap.add_argument('--no-tfrecord-leg', dest='tfrecord_leg', action='store_false')
    return ap.parse_args()


def cpu_baseline(H, W):
    """Oracle (PyTorch-CPU fp32 restatement of the reference step) on ONE image."""
    import config
    from oracle import anchors as oa
    from oracle import net as onet
    from oracle import targets as ot
    from nets.catch_net import CatchNet
    from rod.data import synthetic_boxes
    threads = min(os.cpu_count() or 1, 16)
    torch.set_num_threads(threads)
    cfg = {'train_range': config.train_range.REFINE, 'process_backbone_method': config.process_backbone_method.NONE,
           'deconv_method': config.deconv_method.LEARN_HALF, 'merge_method': config.merge_method.ADD}
    net = CatchNet('mobilenet_v2', cfg, 'cpu', 0)   # parameters only (host copy)
    P = {k: v.detach().clone().requires_grad_(True) for k, v in net.store.params.items()}
    Bf = {k: v.detach().clone() for k, v in net.store.buffers.items()}
    g = torch.Generator().manual_seed(0)
    img = torch.randint(0, 256, (1, H, W, 3), dtype=torch.uint8, generator=g)
    corner, labels, n = synthetic_boxes(1)
    init = oa.init_anchor(6, (H, W))
    chain = oa.feat_sizes((H, W), [s for (_, s, _, _, _) in onet.SPEC])
    anchors = [oa.anchors_one_layer((H, W), chain[t - 1], init[i]) for i, t in enumerate(onet.TAPS)]
    t0 = time.perf_counter()
    x = torch.from_numpy(np.float32(2.0 / 255.0) * img.numpy().astype(np.float32) - np.float32(1.0))
    center = ot.corner_to_center(corner[0, :n[0]])
    gts, _, _, pms = ot.refine_groundtruth(anchors, center, labels[0, :n[0]], config.refine_pos_jac_val_all_layers)
    refine = onet.forward(x, P, Bf, True, moving={})
    loss = 0.
    for l in range(6):
        d = (torch.from_numpy(gts[l][None]) - refine[l]) * torch.from_numpy(pms[l][None]).float()
        ad = d.abs()
        loss = loss + (0.5 * ((ad - 1) * torch.clamp(ad, max=1.0) + ad)).sum()
    loss.backward()
    with torch.no_grad():
        for p in P.values():
            if p.grad is not None:
                p -= 1e-3 * p.grad.clamp(-5, 5)
    dt = time.perf_counter() - t0
    return {'value': round(1.0 / dt, 5), 'unit': 'images/s', 'cores': threads, 'kind': 'port',
            'sample': f'1 image {H}x{W}, one full REFINE train step (targets+fwd+bwd+SGD), oracle fp32 PyTorch-CPU, '
                      f'{dt:.1f} s'}


def cpu_baseline_inference(H, W, rate=0.02):
    """Oracle predict path (BASELINE configs[3] / [4] on the CPU) on ONE image: ALL network in
    eval mode (PyTorch-CPU fp32 restatement), softmax, decode of refine + det against the
    anchors, per-class select / top-k 400 / NMS 0.4 / keep 200 (oracle.post, numpy).  The
    background logit is shifted so that ~`rate` of the class scores pass select_threshold 0.1,
    as in the GPU leg (NMS has real work)."""
    import config
    from oracle import anchors as oa
    from oracle import net as onet
    from oracle import post as op
    from nets.catch_net import CatchNet
    threads = min(os.cpu_count() or 1, 16)
    torch.set_num_threads(threads)
    cfg = {'train_range': config.train_range.ALL, 'process_backbone_method': config.process_backbone_method.NONE,
           'deconv_method': config.deconv_method.LEARN_HALF, 'merge_method': config.merge_method.ADD}
    net = CatchNet('mobilenet_v2', cfg, 'cpu', 0)   # parameters only (host copy)
    P = {k: v.detach().clone() for k, v in net.store.params.items()}
    Bf = {k: v.detach().clone() for k, v in net.store.buffers.items()}
    g = torch.Generator().manual_seed(77)
    img = torch.randint(0, 256, (1, H, W, 3), dtype=torch.uint8, generator=g)
    init = oa.init_anchor(6, (H, W))
    chain = oa.feat_sizes((H, W), [s for (_, s, _, _, _) in onet.SPEC])
    centers = np.concatenate([np.stack(oa.anchor_centers(oa.anchors_one_layer((H, W), chain[t - 1], init[i])),
                                       -1).reshape(-1, 4) for i, t in enumerate(onet.TAPS)]).astype(np.float32)
    t0 = time.perf_counter()
    with torch.no_grad():
        x = torch.from_numpy(np.float32(2.0 / 255.0) * img.numpy().astype(np.float32) - np.float32(1.0))
        refine, det, clf = onet.forward(x, P, Bf, False, all_mode=True)
    t_net = time.perf_counter() - t0
    logits = np.concatenate([c.reshape(1, -1, 11).numpy() for c in clf], 1)
    ro = np.concatenate([r.reshape(1, -1, 4).numpy() for r in refine], 1)
    do = np.concatenate([d.reshape(1, -1, 4).numpy() for d in det], 1)
    lo, hi = -30.0, 30.0          # calibration of the score distribution: not timed
    for _ in range(30):
        mid = 0.5 * (lo + hi)
        lg = logits.copy()
        lg[..., 0] += mid
        e = np.exp(lg - lg.max(-1, keepdims=True))
        if float(((e / e.sum(-1, keepdims=True))[..., 1:] >= 0.1).mean()) > rate:
            lo = mid
        else:
            hi = mid
    logits[..., 0] += hi
    t1 = time.perf_counter()
    e, s_, _ = op.softmax_rows(logits)
    probs = (e / s_).astype(np.float32)
    boxes = op.decode_corner(centers, ro + do)
    scores, _, kept = op.detected_bboxes_vec(probs, boxes, 0.1, 0.4, 400, 200)
    dt = t_net + time.perf_counter() - t1
    return {'value': round(1.0 / dt, 5), 'unit': 'images/s', 'cores': threads, 'kind': 'port',
            'sample': f'1 image {H}x{W}: ALL network eval forward (oracle fp32 PyTorch-CPU, {t_net:.1f} s) + '
                      f'softmax / decode / select / top-k / NMS (oracle numpy, {sum(len(v) for v in kept.values())} '
                      f'boxes kept), {dt:.1f} s'}


def synthetic_jpeg_tfrecord(path, n, H=720, W=1280, seed=5):
    """A TFRecord (dataset/pascalvoc_to_tfrecords.py schema) of n synthetic BDD-shaped frames:
    smooth low-frequency colour fields with mild noise (natural-image-like JPEG size, ~0.1-0.3
    MB at quality 90, unlike i.i.d. noise) and 1..40 boxes each (rod.data.synthetic_boxes)."""
    import io
    from PIL import Image
    from rod import tfrecord
    from rod.data import synthetic_boxes
    rng = np.random.default_rng(seed)
    corner, labels, cnt = synthetic_boxes(n, seed=seed)
    with tfrecord.TFRecordWriter(path) as w:
        for i in range(n):
            small = Image.fromarray(rng.integers(0, 256, (9, 16, 3), dtype=np.uint8))
            img = np.asarray(small.resize((W, H), Image.BICUBIC), np.int16)
            img = np.clip(img + rng.integers(-6, 7, img.shape), 0, 255).astype(np.uint8)
            buf = io.BytesIO()
            Image.fromarray(img).save(buf, format='JPEG', quality=90)
            k = int(cnt[i])
            w.write(tfrecord.encode_detection_example(buf.getvalue(), (H, W, 3), corner[i, :k], labels[i, :k]))


def tfrecord_leg(args, tr, dev, dtype, steps=8, n_img=48):
    """The train.py input path (TFRecord scan + CRC, host JPEG decode on the reference's 4
    reader threads, process_raw_data_train on the GPU) feeding the training step exactly as
    train.py runs it: the source pads the boxes to a fixed count (so the step's HIP graph is
    captured once and replayed whatever each batch's real box count), decodes the next batch on
    a background thread during the current step, and the loop reads each step's losses one
    step late (train._loss_copy / _loss_values).  Reports the host decode rate alone (a
    non-prefetching source) and the fed training rate."""
    step = tr.step_graphed if args.graph else tr.step
    import tempfile
    from rod.dataio import TFRecordSource
    from train import _loss_copy, _loss_values
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, 'bdd100k_train_000.tfrecord')
        t0 = time.perf_counter()
        synthetic_jpeg_tfrecord(path, n_img, args.height, args.width)
        t_write = time.perf_counter() - t0
        nbytes = os.path.getsize(path)
        dec = TFRecordSource([path], args.batch, (args.height, args.width), dev, dtype, train=True, seed=SEED_TF,
                             num_readers=4, prefetch=False)
        dec._host()
        t0 = time.perf_counter()
        for _ in range(steps):   # the host half of a batch: record reads + JPEG decode on the pool + draws
            dec._host()
        t_dec = (time.perf_counter() - t0) / steps
        dec.close()
        src = TFRecordSource([path], args.batch, (args.height, args.width), dev, dtype, train=True, seed=SEED_TF,
                             num_readers=4)
        n_graphs = len(getattr(tr, '_graphs', {}))
        for _ in range(2):
            step(*next(src))
        torch.cuda.synchronize()
        counts = []
        pending = None
        t0 = time.perf_counter()
        for _ in range(steps):
            x, bo, lo, n = next(src)
            counts.append(n)
            losses = step(x, bo, lo, n)
            entry = _loss_copy(losses, 1)
            if pending is not None:
                _loss_values(pending)
            pending = entry
        last = _loss_values(pending)
        torch.cuda.synchronize()
        t_fed = (time.perf_counter() - t0) / steps
        src.close()
        new_graphs = len(getattr(tr, '_graphs', {})) - n_graphs
    real = sorted({int(v) for c in counts for v in c.tolist()})
    return {'metric': 'training images/sec fed from TFRecord (host JPEG decode, 4 reader threads, GPU augmentation)',
            'value': round(args.batch / t_fed, 2), 'unit': 'images/s', 'ms_per_step': round(t_fed * 1e3, 2),
            'host_decode_images_per_s': round(args.batch / t_dec, 2), 'decode_ms_per_batch': round(t_dec * 1e3, 2),
            'num_readers': 4, 'records': n_img, 'mean_record_kb': round(nbytes / n_img / 1024, 1),
            'hip_graph': bool(args.graph), 'graphs_captured': new_graphs, 'gt_padded_to': int(bo.shape[1]),
            'real_box_counts_seen': [real[0], real[-1]] if real else None,
            'write_s': round(t_write, 1), 'loss': round(float(last[0]), 4),
            'data': 'synthetic 1280x720 JPEG frames (smooth colour fields + noise), BDD-shaped boxes'}


def fp32_leg(args, dev, steps=10, warmup=2):
    """BASELINE configs[1] as stated: the REFINE step at 720x1280, batch 8, fp32, one GPU,
    HIP-graph replay."""
    from rod.data import C2_BATCH_SEED, C2_WEIGHT_SEED, synthetic_batch
    from rod.trainer import Trainer
    tr = Trainer((args.height, args.width), args.batch, dtype=torch.float32, device=dev, seed=C2_WEIGHT_SEED)
    batch = synthetic_batch(args.batch, args.height, args.width, dev, seed=C2_BATCH_SEED)
    first = float(tr.step_graphed(*batch)[0].item())   # pinned by tests/test_gpu_fullsize.py (fp32)
    for _ in range(max(warmup, 2) - 1):
        tr.step_graphed(*batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        losses = tr.step_graphed(*batch)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    out = {'metric': 'training images/sec at 1280x720 fp32', 'value': round(args.batch / dt, 3), 'unit': 'images/s',
           'ms_per_step': round(dt * 1e3, 3), 'steps': steps, 'dtype': 'fp32', 'batch': args.batch,
           'loss': round(float(losses[0].item()), 5), 'loss_first_step': round(first, 5), 'hip_graph': True}
    del tr
    torch.cuda.empty_cache()
    return out


SEED_TF = 4242


def dp_overhead_leg(args, dev, dtype, batch, base_ms, steps=10):
    """The data-parallel machinery's cost on one GPU: the headline step (no reducer) against
    the same step with a 1-rank reducer (4 MB buckets):
      'full'        — the N>1 default over RCCL (rod.ddp.make_reducer): the library's
                      communicator, the bucket all-reduces captured on their side stream;
      'sync_bn_full'— the same with SyncBatchNorm (its ~280 rod_allgather calls captured);
      'torch_split' — a torch.distributed reducer: forward + backward replayed, the all-reduce
                      (one per contiguous span) and SGD issued after the replay.
    A 1-rank all-reduce moves no data over xGMI: this prices launch, synchronisation and lost
    overlap, not the link."""
    import socket
    import torch.distributed as dist
    from rod import _abi, ops
    from rod.ddp import GradReducer, make_reducer
    from rod.trainer import Trainer
    from utils import net_tools
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1, device_id=dev)
    out = {'baseline_ms_per_step': round(base_ms, 3), 'world': 1, 'bucket_mb': 4.0, 'steps': steps}
    try:
        from rod.data import C2_WEIGHT_SEED
        for name, mk, kw in (('full', lambda: make_reducer(1, 0), {}),
                             ('sync_bn_full', lambda: make_reducer(1, 0), {'sync_bn': True}),
                             ('torch_split', lambda: GradReducer(1), {})):
            tr = Trainer((args.height, args.width), args.batch, dtype=dtype, device=dev, world_size=1,
                         reducer=mk(), seed=C2_WEIGHT_SEED, **kw)
            for _ in range(3):
                tr.step_graphed(*batch)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                tr.step_graphed(*batch)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            out[name] = {'ms_per_step': round(ms, 3), 'overhead_frac': round(ms / base_ms - 1, 4),
                         'graph_mode': tr.graph_mode(), 'native': bool(tr.reducer.native)}
            del tr
            torch.cuda.empty_cache()
    finally:
        ops.SYNC_BN = None          # Trainer globals: back to the single-process state
        net_tools.HNM_EXCHANGE = None
        _abi.call('rod_rccl_destroy')
        dist.destroy_process_group()
    return out


def inference_fps(args, dev, dtype, batch=32, steps=5, warmup=2, hw=None):
    """BASELINE configs[3] (and [4] with hw=(1080, 1920)): predict.py inference (ALL network,
    eval BN, decode, per-class top-k + NMS), 1 GPU, synthetic batch in HBM, replayed as a HIP
    graph (predict.Predictor).  The random weights get a detector-like score distribution
    first (BatchNorm calibrated, background logit shifted until ~2 % of class scores pass
    select_threshold 0.1), so select / top-k / NMS do real work."""
    import predict
    from rod.data import detector_like_scores, synthetic_batch
    H, W = hw or (args.height, args.width)
    pr = predict.Predictor((H, W), dev, dtype)
    img = synthetic_batch(batch, H, W, dev, seed=77)[0]
    frac = detector_like_scores(pr, img[:4], rate=0.02)
    for _ in range(warmup):
        scores, _ = pr(img)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        scores, _ = pr(img)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kept = sum(int((v > 0).sum()) for v in scores.values())
    return {'metric': 'inference FPS (predict.py path: forward + decode + per-class NMS)',
            'value': round(batch * steps / dt, 2), 'unit': 'images/s', 'img_hw': [H, W], 'batch': batch,
            'steps': steps, 'ms_per_batch': round(dt / steps * 1e3, 3), 'dtype': args.dtype,
            'hip_graph': bool(pr.use_graph), 'selected_frac': round(frac, 4), 'kept_per_image': round(kept / batch, 1),
            'mAP@0.5': None, 'mAP_note': 'no BDD100K data or trained checkpoint on the box (synthetic inputs)'}


def replicated(r, world, dev):
    """An inference leg run by every rank: whole-job images/s over the slowest rank's time."""
    if world == 1:
        return r
    t = torch.tensor([r['ms_per_batch']], device=dev, dtype=torch.float64)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    ms = float(t.item())
    r = dict(r, ms_per_batch=round(ms, 3), value=round(world * r['batch'] * 1e3 / ms, 2), n_gpus=world,
             parallelism=f'{world} replicas (one per GPU, no exchange)')
    return r


NORTH_STAR = ('rod_dw3x3_fwd', 'rod_dw3x3_fwd_rc', 'rod_dw3x3_bwd_fused', 'rod_dw3x3_bwd_fused_pw',
              'rod_dw3x3_bwd_fused_rc', 'rod_dw3x3_bwd_data', 'rod_dw3x3_bwd_filter', 'rod_conv_fwd',
              'rod_conv_fwd_stats', 'rod_conv_wgrad', 'rod_pw_bwd', 'rod_pw_bwd_rc', 'rod_pw_bwd_gred',
              'rod_pw_bwd_gred_rc', 'rod_pw_bwd_gred_dyp', 'rod_bn_bwd_reduce', 'rod_bn_bwd_apply', 'rod_bn_bwd')


def gpu_head_start(ms=120):
    """Park the stream behind a spin kernel (~ms) before the eager probe steps, so the host
    queues their launches ahead of the GPU: every probe event pair then brackets its kernels
    back to back, not host dispatch gaps (an eager step issues in ~21 ms against ~25 ms of GPU
    work, tools/host_time.py, so without this some intervals include waits for the host)."""
    torch.cuda._sleep(int(ms * 1e-3 * 2.4e9))


def kernel_rooflines(tr, batch, steps, dtype):
    """Per-entry rooflines of the north-star kernels (depthwise 3x3, the pointwise / 3x3 GEMMs,
    the BatchNorm backward), timed with HIP events around every call of `steps` extra training
    steps run after the timed region (so the headline number carries no probe overhead).
    Aggregate over all calls of the entry, and its single most expensive call shape.  Every
    other entry is probed too: the step's summed algorithmic bytes / flops (whole-step
    roofline) come from the same steps.  Returns (kernels, step_totals)."""
    from rod import _abi, roofline
    _abi.PROBE.arm('*')
    gpu_head_start()
    for _ in range(steps):
        tr.step(*batch)
    torch.cuda.synchronize()
    _abi.PROBE.disarm()
    agg = _abi.PROBE.table()
    design = _abi.PROBE.design_table()
    by_shape = _abi.PROBE.table(by_shape=True)
    totals = {'cost_model': roofline.COST_MODEL_VERSION,
              'alg_bytes_per_step': sum(v[2] for v in agg.values()) // steps,
              'alg_flops_per_step': sum(v[3] for v in agg.values()) // steps,
              'design_bytes_per_step': sum(design.values()) // steps,
              'launch_entries_per_step': sum(v[0] for v in agg.values()) // steps,
              'probed_kernel_ms_per_step': round(sum(v[1] for v in agg.values()) / steps, 3)}
    peak_tf = roofline.MI355X_BF16_PEAK_TFLOPS if dtype == torch.bfloat16 else roofline.MI355X_F32_PEAK_TFLOPS
    out = {}
    for name in NORTH_STAR:
        if name not in agg:
            continue
        n, ms, b, fl = agg[name]
        top = max(((k, v) for k, v in by_shape.items() if k[0] == name), key=lambda kv: kv[1][1])
        tn, tms, tb, tfl = top[1]
        gbs, tgbs = b / ms / 1e6, tb / tms / 1e6
        out[name] = {'launches_per_step': n // steps, 'ms_per_step': round(ms / steps, 3),
                     'alg_GBps': round(gbs, 1), 'hbm_frac': round(gbs / roofline.MI355X_HBM_PEAK_GBS, 4),
                     'alg_TFLOPs': round(fl / ms / 1e9, 2), 'mfma_frac': round(fl / ms / 1e9 / peak_tf, 5),
                     'top_call': {'args': list(top[0][1]), 'avg_us': round(1e3 * tms / tn, 1),
                                  'alg_GBps': round(tgbs, 1), 'hbm_frac': round(tgbs / roofline.MI355X_HBM_PEAK_GBS, 4),
                                  'alg_TFLOPs': round(tfl / tms / 1e9, 2)}}
        if design.get(name, b) != b:
            out[name]['design_GBps'] = round(design[name] / ms / 1e6, 1)
    return out, totals


def main():
    args = parse()
    # stdout carries exactly ONE line, the JSON result: anything else written to fd 1 (RCCL's
    # version banner at communicator init, library prints) goes to stderr
    json_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # RCCL ('nccl') is the product path; ROD_DIST_BACKEND=gloo rehearses the N>1 path with
    # several ranks sharing the GPUs of a smaller box (device = LOCAL_RANK mod device count)
    backend = os.environ.get('ROD_DIST_BACKEND', 'nccl')
    if world > 1:
        local = local % torch.cuda.device_count() if backend != 'nccl' else local
        torch.cuda.set_device(local)
        if backend == 'nccl':
            torch.distributed.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            torch.distributed.init_process_group(backend)
    dev = torch.device('cuda', local)
    import config
    from rod import _abi, roofline
    from rod.data import C2_BATCH_SEED, C2_WEIGHT_SEED, SEED, synthetic_batch
    from rod.trainer import Trainer

    dtype = torch.bfloat16 if args.dtype == 'bf16' else torch.float32
    tr_range = config.train_range.REFINE if args.train_range == 'REFINE' else config.train_range.ALL
    reducer = None
    if world > 1:
        # bucketed all-reduce launched during backward: over RCCL the library's communicator on a
        # side stream (the whole step captured, 'full'); gloo (rehearsal): torch.distributed
        from rod.ddp import make_reducer
        reducer = make_reducer(world, rank)
    tr = Trainer((args.height, args.width), args.batch, dtype=dtype, train_range=tr_range, device=dev,
                 world_size=world, reducer=reducer, fix_refine=args.fix_refine, sync_bn=args.sync_bn,
                 seed=C2_WEIGHT_SEED)
    # rank 0's batch and the initial weights are the ones tests/test_gpu_fullsize.py pins
    batch = synthetic_batch(args.batch, args.height, args.width, dev, seed=C2_BATCH_SEED + rank)
    source = None
    if args.augment:
        from rod.dataio import AugmentedSource
        source = AugmentedSource(args.batch, (args.height, args.width), dev, dtype, seed=SEED + rank, n_distinct=2)
    next_batch = (lambda: next(source)) if source is not None else (lambda: batch)
    # Trainer.graph_mode decides what the graph holds: the whole step (N=1, or N>1 over RCCL
    # through the library's communicator), forward + backward only ('split': the gloo
    # rehearsal), or nothing (gloo with collectives inside the step)
    use_graph = args.graph and tr.graph_mode() != 'eager'
    step = tr.step_graphed if use_graph else tr.step

    # graphed: the capture happens on the second call (after one eager set-up step), so at
    # least two untimed calls run before the timed region whatever --warmup says
    first_loss = None
    for i in range(max(args.warmup, 2) if use_graph else args.warmup):
        lw = step(*next_batch())
        if i == 0:   # the first step's loss: from the initial weights, pinned against the fp64
            first_loss = float(lw[0].item())   # oracle by tests/test_gpu_fullsize.py (bf16, 720p, b8)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    probe_set = [p for p in args.probe.split(',') if p]
    _abi.PROBE.arm('*' if args.probe_table else probe_set)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        losses = step(*next_batch())
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    _abi.PROBE.disarm()
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())

    table, design = _abi.PROBE.table(), _abi.PROBE.design_table()
    probe_steps = args.steps
    if use_graph:
        # a replayed graph makes no host calls to time: the dominant kernel's rooflines come
        # from two eager steps after the timed region (same kernels, same arguments)
        _abi.PROBE.arm(probe_set)
        gpu_head_start()
        for _ in range(2):
            tr.step(*next_batch())
        torch.cuda.synchronize()
        _abi.PROBE.disarm()
        table, design, probe_steps = _abi.PROBE.table(), _abi.PROBE.design_table(), 2
    n_launch, ms, byts, flops = 0, 0.0, 0, 0
    for p in probe_set:
        e = table.get(p, (0, 0.0, 0, 0))
        n_launch, ms, byts, flops = n_launch + e[0], ms + e[1], byts + e[2], flops + e[3]
    dbytes = sum(design.get(p, 0) for p in probe_set)
    loss_val = float(losses[0].item())
    kernels = step_totals = None
    if args.kernel_steps > 0 and world == 1:
        kernels, step_totals = kernel_rooflines(tr, batch, args.kernel_steps, dtype)
    tf_leg = None
    if args.tfrecord_leg and world == 1:
        tf_leg = tfrecord_leg(args, tr, dev, dtype)
    fp32 = None
    if args.fp32_leg and world == 1 and dtype == torch.bfloat16:
        fp32 = fp32_leg(args, dev)
    dp_over = None
    if args.dp_leg and world == 1 and args.graph and tr_range is config.train_range.REFINE:
        dp_over = dp_overhead_leg(args, dev, dtype, batch, base_ms=elapsed / args.steps * 1e3)
    if args.probe_table and rank == 0:
        # per-entry live timing (every call bracketed by events; the step itself is slower
        # in this mode, so ms_per_step of such a run is not a bench number)
        with open(args.probe_table, 'w') as f:
            rows = []
            for name, (n, t, b, fl) in sorted(table.items(), key=lambda kv: -kv[1][1]):
                rows.append({'entry': name, 'calls_per_step': n / args.steps, 'ms_per_step': t / args.steps,
                             'avg_us': 1e3 * t / n, 'alg_GBps': b / max(t, 1e-9) / 1e6,
                             'alg_TFLOPs': fl / max(t, 1e-9) / 1e9})
            calls = []
            for (name, shp), (n, t, b, fl) in sorted(_abi.PROBE.table(by_shape=True).items(),
                                                     key=lambda kv: -kv[1][1])[:120]:
                calls.append({'entry': name, 'args': list(shp), 'calls_per_step': n / args.steps,
                              'avg_us': 1e3 * t / n, 'alg_GBps': b / max(t, 1e-9) / 1e6,
                              'alg_TFLOPs': fl / max(t, 1e-9) / 1e9})
            json.dump({'cost_model': roofline.COST_MODEL_VERSION, 'entries': rows, 'top_calls': calls}, f, indent=1)

    # inference legs (configs[3], configs[4]): at N > 1 every rank runs the same predict path on
    # its own batch (inference does not shard: replicas); the aggregate is all ranks' images over
    # the slowest rank's time
    inf = inf1080 = None
    if args.inference:
        inf = replicated(inference_fps(args, dev, dtype), world, dev)
        if args.inference_1080:   # configs[4]: 1920x1080 bf16, fused inverted-residual blocks
            inf1080 = replicated(inference_fps(args, dev, dtype, batch=8, hw=(1080, 1920)), world, dev)
    if rank == 0:
        per_launch_ms = ms / max(n_launch, 1)
        achieved_gbs = byts / max(ms, 1e-9) / 1e6
        achieved_tf = flops / max(ms, 1e-9) / 1e9
        peak_tf = roofline.MI355X_BF16_PEAK_TFLOPS if dtype == torch.bfloat16 else roofline.MI355X_F32_PEAK_TFLOPS
        # bound: whichever roof the kernel's aggregate arithmetic intensity meets first
        ai = flops / max(byts, 1)
        ridge = peak_tf * 1e12 / (roofline.MI355X_HBM_PEAK_GBS * 1e9)
        if ai < ridge:
            rl = {'bound': 'hbm', 'achieved': round(achieved_gbs, 1), 'peak': roofline.MI355X_HBM_PEAK_GBS,
                  'unit': 'GB/s', 'frac': round(achieved_gbs / roofline.MI355X_HBM_PEAK_GBS, 4)}
        else:
            rl = {'bound': 'mfma', 'achieved': round(achieved_tf, 2), 'peak': peak_tf, 'unit': 'TFLOP/s',
                  'frac': round(achieved_tf / peak_tf, 4)}
        traffic, tsrc, pmc_lps, tj = None, None, None, {}
        if args.traffic and os.path.exists(args.traffic):
            tj = json.load(open(args.traffic))
            tes = [tj.get('entries', {}).get(p) for p in probe_set]
            if all(te is not None for te in tes) and \
                    tj.get('config') == [args.train_range, args.batch, args.height, args.width, args.dtype]:
                # per launch of the family: total PMC bytes of its entries / their launches
                traffic = round(sum(te['bytes_per_launch'] * te['launches'] for te in tes) /
                                max(1, sum(te['launches'] for te in tes)))
                tsrc = os.path.relpath(args.traffic, ROOT)
                # the PMC run's launches of the family per profiled step: must equal the probe's
                if all(te.get('launches_per_step') is not None for te in tes):
                    pmc_lps = sum(te['launches_per_step'] for te in tes)
        rl.update({'traffic': traffic, 'traffic_unit': 'bytes/launch (HBM, PMC)', 'traffic_source': tsrc,
                   'traffic_launches_per_step': pmc_lps,
                   'cost_model': roofline.COST_MODEL_VERSION,
                   'alg_bytes_per_launch': byts // max(n_launch, 1), 'kernel': args.probe.replace(',', ' + '),
                   'launches_per_step': n_launch // max(probe_steps, 1),
                   'avg_launch_us': round(per_launch_ms * 1e3, 2), 'alg_bytes_per_step': byts // max(probe_steps, 1),
                   'alg_flops_per_step': flops // max(probe_steps, 1),
                   # the bytes the design moves (rod.roofline.design_bytes): for the fused depthwise
                   # backward + the re-read of (dz, y) of its output BatchNorm (the reduce pass
                   # read them first); for the BatchNorm family reduce 2 + apply 3 passes
                   'design_bytes_per_step': dbytes // max(probe_steps, 1),
                   'design_GBps': round(dbytes / max(ms, 1e-9) / 1e6, 1),
                   'traffic_over_alg': round(traffic / max(byts // max(n_launch, 1), 1), 3) if traffic else None,
                   'traffic_over_design': round(traffic / max(dbytes // max(n_launch, 1), 1), 3) if traffic else None})
        step_rl = None
        if step_totals is not None:
            # whole step: every call's algorithmic bytes over the timed ms per step
            sgbs = step_totals['alg_bytes_per_step'] / (elapsed / args.steps) / 1e9
            step_rl = dict(step_totals, achieved_GBps=round(sgbs, 1), peak=roofline.MI355X_HBM_PEAK_GBS,
                           frac=round(sgbs / roofline.MI355X_HBM_PEAK_GBS, 4),
                           alg_TFLOPs=round(step_totals['alg_flops_per_step'] / (elapsed / args.steps) / 1e12, 2),
                           note='sum of algorithmic bytes of every librod call of a step (rod.roofline) / the timed '
                                'ms_per_step; probed over eager steps after the timed region')
            if tsrc is not None and tj.get('all_bytes_per_step'):
                # the PMC passes' whole-step HBM bytes (every kernel), and the part the entries claim
                step_rl.update(pmc_bytes_per_step=round(tj['all_bytes_per_step']),
                               pmc_attributed_bytes_per_step=round(tj['attributed_bytes_per_step']),
                               pmc_over_alg=round(tj['all_bytes_per_step'] / max(step_totals['alg_bytes_per_step'], 1), 3))
        imgs = args.batch * world * args.steps
        out = {
            'metric': 'training images/sec at 1280x720 bf16' if dtype == torch.bfloat16 else
                      'training images/sec at 1280x720 fp32',
            'value': round(imgs / elapsed, 3), 'unit': 'images/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': args.dtype, 'data': 'synthetic',
            'config': {'workload': f'{args.train_range} train step (train.py), MobileNet-v2 RefineDet, '
                                   f'{args.height}x{args.width}, {args.batch} images/GPU',
                       'global_batch': args.batch * world, 'img_hw': [args.height, args.width],
                       'train_range': args.train_range, 'parallelism': f'dp{world}',
                       'augment': bool(args.augment), 'hip_graph': bool(use_graph),
                       'graph_mode': tr.graph_mode() if use_graph else 'eager',
                       **({'dist_backend': 'rccl' if backend == 'nccl' else backend,
                           'batchnorm': 'sync (global batch)' if args.sync_bn else 'per rank'} if world > 1 else {}),
                       **({} if args.train_range == 'REFINE' else {'fix_refine': args.fix_refine})},
            'loss': round(loss_val, 5), 'loss_first_step': round(first_loss, 5) if first_loss is not None else None,
            'roofline': rl,
        }
        if step_rl is not None:
            out['step_roofline'] = step_rl
        if kernels is not None:
            out['kernels'] = kernels
        if fp32 is not None:
            out['training_fp32'] = fp32
        if tf_leg is not None:
            out['tfrecord'] = tf_leg
        if dp_over is not None:
            out['dp_overhead'] = dp_over
        if args.cpu_baseline and world == 1:
            if inf is not None:
                inf['cpu_baseline'] = cpu_baseline_inference(args.height, args.width)
            if inf1080 is not None:
                inf1080['cpu_baseline'] = cpu_baseline_inference(1080, 1920)
        if inf is not None:
            out['inference'] = inf
        if inf1080 is not None:
            out['inference_1080p'] = inf1080
        if args.cpu_baseline and world == 1:
            out['cpu_baseline'] = cpu_baseline(args.height, args.width)
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + '\n').encode())
    if world > 1:
        if getattr(reducer, 'native', False):
            _abi.call('rod_rccl_destroy')
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
