"""Roofline report for BASELINE configs[4] (1920x1080 bf16, the fused depthwise + pointwise
inverted-residual blocks, predict.py path) — VERDICT r1 item 5.

Two steps, both on the GPU box:
  python tools/c5_report.py probe --res 1080 --batch 8 --out P.json
      eager Predictor iterations with every librod call bracketed by HIP events on its stream:
      per entry launches / ms / algorithmic bytes and flops per iteration (rod/roofline.py)
  python tools/c5_report.py pmc P.json FETCH.csv WRITE.csv MFMA.csv --out R.json
      adds the rocprofv3 PMC passes of `tools/predict_bench.py --no-graph` (separate runs:
      FETCH_SIZE / WRITE_SIZE / SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE) per kernel family:
      measured HBM bytes (FETCH_SIZE x2: the gfx950 16-byte-lane read correction of
      MI355X_MICROARCH.md; KiB units), MFMA-busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
      GRBM_GUI_ACTIVE / 8 XCDs), and each family's roofline bound min(MFMA peak, AI x HBM peak).
      Only the dispatches of the last --runs passes count (from the --runs-th last
      normalize_image launch: predict_bench's 2 warm-up + --iters passes, default 2 + 3): before
      them predict_bench calibrates the score distribution on 4
      images (detector_like_scores), ~15 smaller passes whose dispatches the rocprofv3 CSVs hold
      too — averaged in, they pulled the round-4 report's traffic/alg below 1 (0.78)."""
import argparse
import collections
import csv
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'))

# entry -> kernel-name substrings of every kernel it launches (PMC attribution); rod_conv_fwd's
# 1x1 streaming, stem and split-K combine kernels included (rod_conv_fwd_bnact shares them)
FAMILIES = {'rod_ir_block_fwd': ('ir_block_fwd_kernel',),
            'rod_conv_fwd': ('conv_fwd_kernel', 'pw_stream_kernel', 'stem_fwd_mfma_kernel', 'stem_conv_fwd_kernel',
                             'splitk_combine_kernel'),
            'rod_dw3x3_fwd': ('dw3x3_fwd_kernel', 'dw3x3_fwd_lx_kernel'),
            'rod_dw3x3_fwd_rc': ('dw3x3_fwd_rc_kernel',), 'rod_bn_apply': ('bn_apply_kernel',)}


def probe(a):
    import torch
    import predict
    from rod import _abi
    from rod.data import detector_like_scores, synthetic_batch
    H, W = (720, 1280) if a.res == 720 else (1080, 1920)
    dev = torch.device('cuda')
    pr = predict.Predictor((H, W), dev, torch.bfloat16)
    pr.use_graph = False
    img = synthetic_batch(a.batch, H, W, dev, seed=77)[0]
    detector_like_scores(pr, img[:4], rate=0.02)
    for _ in range(2):
        pr(img)
    torch.cuda.synchronize()
    _abi.PROBE.arm('*')
    t0 = time.perf_counter()
    for _ in range(a.iters):
        pr(img)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    _abi.PROBE.disarm()
    rows = {}
    for name, (n, ms, b, fl) in _abi.PROBE.table().items():
        rows[name] = {'launches': n / a.iters, 'ms': ms / a.iters, 'alg_bytes': b / a.iters, 'alg_flops': fl / a.iters}
    by_shape = _abi.PROBE.table(by_shape=True)
    shapes = [{'entry': k[0], 'args': list(k[1]), 'launches': v[0] / a.iters, 'ms': v[1] / a.iters}
              for k, v in by_shape.items() if k[0] == 'rod_ir_block_fwd']
    # the conv family per call shape (scalar args: M / N, H, W, Cin, Cout, ks ...), slowest first
    convs = sorted(({'entry': k[0], 'args': list(k[1]), 'launches': v[0] / a.iters, 'ms': v[1] / a.iters,
                     'alg_GBps': v[2] / max(v[1], 1e-9) * 1e-6, 'alg_TFLOPs': v[3] / max(v[1], 1e-9) * 1e-9}
                    for k, v in by_shape.items() if k[0] in ('rod_conv_fwd', 'rod_conv_fwd_bnact')),
                   key=lambda r: -r['ms'])
    out = {'img_hw': [H, W], 'batch': a.batch, 'iters': a.iters, 'eager_ms_per_batch': dt * 1e3,
           'entries': rows, 'ir_block_calls': shapes, 'conv_calls': convs}
    json.dump(out, open(a.out, 'w'), indent=1)
    for r in convs[:25]:
        print('%-20s %-60s x%.0f %7.3f ms %7.0f GB/s %6.1f TF' % (r['entry'], r['args'], r['launches'], r['ms'],
                                                               r['alg_GBps'], r['alg_TFLOPs']))
    print(json.dumps({k: round(v['ms'], 3) for k, v in sorted(rows.items(), key=lambda kv: -kv[1]['ms'])[:8]}))


def per_dispatch(path, counters):
    """{dispatch id: (kernel name, {counter: value})} of the counters asked for."""
    import gzip
    f = gzip.open(path, 'rt') if path.endswith('.gz') else open(path)
    d = {}
    for r in csv.DictReader(f):
        if r['Counter_Name'] in counters:
            k = int(r.get('Dispatch_Id') or r.get('Correlation_Id'))
            d.setdefault(k, (r['Kernel_Name'], collections.defaultdict(float)))[1][r['Counter_Name']] += \
                float(r['Counter_Value'])
    return d


def family_sum(d, subs, runs):
    """Counter sums over the dispatches of the last `runs` predict passes (each pass starts with
    its one normalize_image launch) whose kernel name contains one of subs."""
    starts = sorted(k for k, (name, _) in d.items() if 'normalize_image' in name)
    first = starts[-runs] if len(starts) >= runs else 0
    tot = collections.defaultdict(float)
    n = 0
    for k, (name, cs) in d.items():
        if k >= first and any(s in name for s in subs):
            n += 1
            for c, v in cs.items():
                tot[c] += v
    return tot, n


def pmc(a):
    from rod import roofline
    P = json.load(open(a.probe))
    fetch = per_dispatch(a.fetch, {'FETCH_SIZE'})
    write = per_dispatch(a.write, {'WRITE_SIZE'})
    mfma = per_dispatch(a.mfma, {'SQ_VALU_MFMA_BUSY_CYCLES', 'GRBM_GUI_ACTIVE'})
    peak_tf, peak_bw = roofline.MI355X_BF16_PEAK_TFLOPS, roofline.MI355X_HBM_PEAK_GBS
    rep = {'config': 'BASELINE configs[4]: predict.py path, %dx%d, batch %d, bf16' %
                     (P['img_hw'][1], P['img_hw'][0], P['batch']),
           'method': __doc__.split('\n\n')[1].strip(), 'families': {}}
    for entry, sub in FAMILIES.items():
        e = P['entries'].get(entry)
        if entry == 'rod_conv_fwd' and P['entries'].get('rod_conv_fwd_bnact'):
            # the inference BatchNorm epilogue (ABI 21) runs the same conv_fwd_kernel family: one
            # family of launches for both entries
            b = P['entries']['rod_conv_fwd_bnact']
            e = {k: (e or {}).get(k, 0) + b[k] for k in ('launches', 'ms', 'alg_bytes', 'alg_flops')}
        if not e:
            continue
        f, nfd = family_sum(fetch, sub, a.runs)
        w, _ = family_sum(write, sub, a.runs)
        m, _ = family_sum(mfma, sub, a.runs)
        if nfd == 0:
            continue
        rd = 2.0 * 1024 * f['FETCH_SIZE'] / a.runs
        wr = 1024.0 * w['WRITE_SIZE'] / a.runs
        busy, gui = m['SQ_VALU_MFMA_BUSY_CYCLES'], m['GRBM_GUI_ACTIVE']
        t = e['ms'] * 1e-3
        ai = e['alg_flops'] / max(e['alg_bytes'], 1)
        bound_tf = min(peak_tf, ai * peak_bw / 1e3)
        ach_tf = e['alg_flops'] / t / 1e12
        rep['families'][entry] = {
            'launches_per_iter': e['launches'], 'ms_per_iter': round(e['ms'], 3),
            'alg_GB_per_iter': round(e['alg_bytes'] / 1e9, 4), 'hbm_GB_per_iter_pmc': round((rd + wr) / 1e9, 4),
            'traffic_over_alg': round((rd + wr) / max(e['alg_bytes'], 1), 3),
            'alg_GBps': round(e['alg_bytes'] / t / 1e9, 1), 'hbm_GBps_pmc': round((rd + wr) / t / 1e9, 1),
            'hbm_frac_pmc': round((rd + wr) / t / 1e9 / peak_bw, 4),
            'alg_TFLOPs': round(ach_tf, 2), 'mfma_frac_flops': round(ach_tf / peak_tf, 4),
            'mfma_busy_pmc': round(busy / max(1024 * gui / 8.0, 1), 4),
            'ai_flop_per_byte': round(ai, 1), 'roofline_bound': 'mfma' if ai * peak_bw / 1e3 >= peak_tf else 'hbm',
            'roofline_TFLOPs': round(bound_tf, 1), 'frac_of_roofline': round(ach_tf / bound_tf, 4)}
    json.dump(rep, open(a.out, 'w'), indent=1)
    for k, v in rep['families'].items():
        print(k, json.dumps(v))


def main():
    ap = argparse.ArgumentParser()
    sp = ap.add_subparsers(dest='cmd', required=True)
    p = sp.add_parser('probe')
    p.add_argument('--res', type=int, default=1080)
    p.add_argument('--batch', type=int, default=8)
    p.add_argument('--iters', type=int, default=5)
    p.add_argument('--out', required=True)
    q = sp.add_parser('pmc')
    q.add_argument('probe')
    q.add_argument('fetch')
    q.add_argument('write')
    q.add_argument('mfma')
    q.add_argument('--out', required=True)
    q.add_argument('--runs', type=int, default=5, help="predict_bench's passes at the measured batch (2 + --iters)")
    a = ap.parse_args()
    probe(a) if a.cmd == 'probe' else pmc(a)


if __name__ == '__main__':
    main()
