"""Drop-in for the reference's utils/tf_extended (bboxes, metrics, math, tensors).

Evaluation bookkeeping (matching, TP/FP accumulation, precision/recall, VOC AP) runs on the
host in numpy, as the reference pins it to the CPU (evaluate.py:146, 164); the per-class
sort + NMS runs as the rod_select_topk_nms kernel (utils.net_tools.detected_bboxes).
"""
from utils.tf_extended.bboxes import *  # noqa: F401,F403
from utils.tf_extended.math import *  # noqa: F401,F403
from utils.tf_extended.metrics import *  # noqa: F401,F403
from utils.tf_extended.tensors import *  # noqa: F401,F403
