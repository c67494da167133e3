"""Box-format helpers and logger (reference utils/common_tools.py:11-56).

Both conversions run as the rod_boxes_convert kernel on [..., 4] fp32 device tensors.
"""
import logging

import torch

from rod import ops

logging.basicConfig(level=logging.INFO, format='%(asctime)s - %(levelname)s - %(message)s')
logger = logging.getLogger(__name__)


def centerBboxes_2_cornerBboxes(center_bboxes: torch.Tensor) -> torch.Tensor:
    """[yc, xc, h, w] -> [ymin, xmin, ymax, xmax] (common_tools.py:16-35)."""
    return ops.boxes_convert(center_bboxes, to_center=False)


def cornerBboxes_2_centerBboxes(corner_bboxes: torch.Tensor) -> torch.Tensor:
    """[ymin, xmin, ymax, xmax] -> [yc, xc, h, w] (common_tools.py:38-56)."""
    return ops.boxes_convert(corner_bboxes, to_center=True)
