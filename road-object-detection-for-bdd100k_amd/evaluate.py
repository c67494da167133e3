"""mAP evaluation CLI — drop-in for the reference's evaluate.py (flags 37-69, flow 86-241).

ALL-mode network in inference mode -> softmax + decode(refine_out + det_out) ->
detected_bboxes (per-class select / top-k / NMS, one kernel) -> TP/FP matching against the
ground truth -> streaming TP/FP arrays -> VOC07 / VOC12 AP per class and their mean, over
ceil(3000 / batch_size) batches (evaluate.py:219).  Matching and AP are host code, as the
reference pins them to the CPU (evaluate.py:146, 164).
"""
import argparse
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import config  # noqa: E402
from utils.common_tools import logger  # noqa: E402


def str2bool(v):
    return v if isinstance(v, bool) else str(v).lower() in ('1', 'true', 't', 'yes', 'y')


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument('--backbone_name', default='mobilenet_v2')
    ap.add_argument('--num_readers', type=int, default=4)
    ap.add_argument('--num_preprocessing_threads', type=int, default=4)
    ap.add_argument('--checkpoint_path', default='checkpoint/')
    ap.add_argument('--eval_dir', default='evaluation/')
    ap.add_argument('--batch_size', type=int, default=1)
    ap.add_argument('--select_threshold', type=float, default=0.3)
    ap.add_argument('--select_top_k', type=int, default=400)
    ap.add_argument('--keep_top_k', type=int, default=200)
    ap.add_argument('--nms_threshold', type=float, default=0.4)
    ap.add_argument('--matching_threshold', type=float, default=0.5)
    ap.add_argument('--gpu_memory_fraction', type=float, default=0.8)
    # additions
    ap.add_argument('--num_images', type=int, default=3000, help='evaluate.py:219 hard-codes 3000')
    ap.add_argument('--img_height', type=int, default=config.img_size[0])
    ap.add_argument('--img_width', type=int, default=config.img_size[1])
    ap.add_argument('--dtype', default='fp32', choices=['fp32', 'bf16'])
    ap.add_argument('--dataset_dir', default='./dataset/bdd100k_TfRecord/')
    ap.add_argument('--synthetic', type=str2bool, default=False,
                    help='run on synthetic BDD-shaped batches (no dataset needed); results are not real '
                         'metrics.  Without it a missing dataset or checkpoint is an error')
    return ap.parse_args(argv)


def latest_checkpoint(path, backbone):
    """A torch checkpoint (train.py writes <train_dir>/<backbone>.model) or a TF-1.x tensor
    bundle (<prefix>.index + .data-*), as a directory or a file prefix."""
    from rod.checkpoint import exists
    if os.path.isdir(path):
        cand = os.path.join(path, backbone + '.model')
        if exists(cand):
            return cand
        from rod.checkpoint import tf_latest_checkpoint
        return tf_latest_checkpoint(path)
    return path if exists(path) else None


def main(argv=None):
    F = parse(argv)
    logger.info('Asserting parameters')
    assert F.backbone_name in config.supported_backbone_name
    from nets.catch_net import CatchNet, factory
    from rod.dataio import make_source, network_input
    from utils import net_tools
    from utils.common_tools import cornerBboxes_2_centerBboxes  # noqa: F401
    import utils.tf_extended as tfe

    dev = torch.device('cuda', 0)
    config.img_size = (F.img_height, F.img_width)
    dtype = torch.bfloat16 if F.dtype == 'bf16' else torch.float32
    layer_n = len(config.extract_feat_name[F.backbone_name])
    anchors_all = net_tools.anchors_all_layer(config.img_size, config.feat_sizes(config.img_size, F.backbone_name),
                                              net_tools.init_anchor(layer_n))
    config_dict = {'process_backbone_method': config.process_backbone_method.NONE,
                   'deconv_method': config.deconv_method.LEARN_HALF,
                   'merge_method': config.merge_method.ADD, 'train_range': config.train_range.ALL}
    logger.info('Building model, using backbone---%s' % F.backbone_name)
    net = CatchNet(F.backbone_name, config_dict, dev)
    ckpt = latest_checkpoint(F.checkpoint_path, F.backbone_name)
    if ckpt is not None:
        from rod.checkpoint import load_variables
        load_variables(net.store, ckpt)
        logger.info('Evaluating %s' % ckpt)
    elif F.synthetic:
        logger.warning('--synthetic: no checkpoint at %r, evaluating randomly initialised weights',
                       F.checkpoint_path)
    else:   # tf.train.latest_checkpoint(...) -> None makes the reference's restore fail
        raise FileNotFoundError('no checkpoint under %r (evaluate.py:221-224)' % F.checkpoint_path)
    logger.info('Building data pileline, using dataset---%s' % 'bdd100k_train')
    source = make_source(F.dataset_dir, F.batch_size, config.img_size, dev, split='train', synthetic=F.synthetic,
                         dtype=dtype, num_readers=F.num_readers, max_images=F.num_images)

    num_batches = math.ceil(F.num_images / float(F.batch_size))
    state = None
    classes = list(range(1, config.total_obj_n))
    start = time.time()
    with torch.no_grad():
        for _ in range(num_batches):
            img, gboxes, glabels, gn = next(source)
            x = network_input(img, dtype)
            refine_out, det_out, clf_out = factory(x, F.backbone_name, False, config_dict, dtype,
                                                   net=net).get_output()
            probs = net_tools.class_probabilities(clf_out)
            boxes = net_tools.decode_all_layers(anchors_all, refine_out, det_out, to_corner=True)
            rscores, rbboxes = net_tools.detected_bboxes(probs, boxes, select_threshold=F.select_threshold,
                                                         nms_threshold=F.nms_threshold, top_k=F.select_top_k,
                                                         keep_top_k=F.keep_top_k)
            rs = {c: v.cpu().numpy() for c, v in rscores.items()}
            rb = {c: v.cpu().numpy() for c, v in rbboxes.items()}
            gl, gb, gcount = glabels.cpu().numpy(), gboxes.cpu().numpy(), gn.cpu().numpy()
            n_g, tp, fp, _ = tfe.bboxes_matching_batch(classes, rs, rb, gl, gb, np.zeros_like(gl),
                                                       matching_threshold=F.matching_threshold, gt_counts=gcount)
            state = tfe.streaming_tp_fp_arrays(n_g, tp, fp, rs, state=state)
    aps07, aps12 = {}, {}
    for c in classes:
        prec, rec = tfe.precision_recall(*state[c].value())
        aps07[c] = tfe.average_precision_voc07(prec, rec)
        aps12[c] = tfe.average_precision_voc12(prec, rec)
        logger.info('AP_VOC07/%d %.6f  AP_VOC12/%d %.6f' % (c, aps07[c], c, aps12[c]))
    mAP07 = sum(aps07.values()) / len(aps07)
    mAP12 = sum(aps12.values()) / len(aps12)
    if F.synthetic:
        logger.warning('--synthetic: the AP values below are over synthetic ground truth, not a BDD100K result')
    print('AP_VOC07/mAP[%s]' % mAP07)
    print('AP_VOC12/mAP[%s]' % mAP12)
    elapsed = time.time() - start
    print('Time spent : %.3f seconds.' % elapsed)
    print('Time spent per BATCH: %.3f seconds.' % (elapsed / num_batches))
    os.makedirs(F.eval_dir, exist_ok=True)
    with open(os.path.join(F.eval_dir, 'eval.json'), 'w') as f:
        import json
        json.dump({'AP_VOC07': aps07, 'AP_VOC12': aps12, 'mAP_VOC07': mAP07, 'mAP_VOC12': mAP12,
                   'num_batches': num_batches, 'seconds': elapsed, 'synthetic': bool(F.synthetic),
                   'checkpoint': ckpt}, f)
    return mAP07, mAP12


if __name__ == '__main__':
    main()
