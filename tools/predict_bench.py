"""Run the predict.py inference path (Predictor: forward + decode + per-class NMS, HIP-graph
replay) on a synthetic batch with a detector-like score distribution, for rocprofv3 kernel
traces of configs[3] / configs[4].
Usage: python tools/predict_bench.py [--res 720|1080] [--batch 32] [--iters 10] [--no-graph]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--res', type=int, default=720)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--no-graph', action='store_true')
    a = ap.parse_args()
    import predict
    from rod.data import detector_like_scores, synthetic_batch
    H, W = (720, 1280) if a.res == 720 else (1080, 1920)
    dev = torch.device('cuda')
    pr = predict.Predictor((H, W), dev, torch.bfloat16)
    pr.use_graph = not a.no_graph
    img = synthetic_batch(a.batch, H, W, dev, seed=77)[0]
    frac = detector_like_scores(pr, img[:4], rate=0.02)
    for _ in range(2):
        pr(img)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        pr(img)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    print(json.dumps({'img_hw': [H, W], 'batch': a.batch, 'graph': pr.use_graph, 'ms_per_batch': round(dt * 1e3, 3),
                      'images_per_s': round(a.batch / dt, 1), 'selected_frac': round(frac, 4)}), flush=True)


if __name__ == '__main__':
    main()
