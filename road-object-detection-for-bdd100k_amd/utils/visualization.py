"""Detection drawing for predict.py (reference utils/net_tools.py:761-1106, the box / mask /
keypoint overlay helpers predict.py:151-196 calls).  Host-side PIL on uint8 RGB arrays; the
functions keep the reference's names, arguments and in-place behaviour.  Fonts: Arial when the
host has it, PIL's built-in bitmap font otherwise (as the reference falls back)."""
from __future__ import annotations

import collections

import numpy as np
from PIL import Image, ImageColor, ImageDraw, ImageFont

STANDARD_COLORS = [
    'AliceBlue', 'Chartreuse', 'Aqua', 'Aquamarine', 'Azure', 'Beige', 'Bisque', 'BlanchedAlmond', 'BlueViolet',
    'BurlyWood', 'CadetBlue', 'AntiqueWhite', 'Chocolate', 'Coral', 'CornflowerBlue', 'Cornsilk', 'Crimson', 'Cyan',
    'DarkCyan', 'DarkGoldenRod', 'DarkGrey', 'DarkKhaki', 'DarkOrange', 'DarkOrchid', 'DarkSalmon', 'DarkSeaGreen',
    'DarkTurquoise', 'DarkViolet', 'DeepPink', 'DeepSkyBlue', 'DodgerBlue', 'FireBrick', 'FloralWhite', 'ForestGreen',
    'Fuchsia', 'Gainsboro', 'GhostWhite', 'Gold', 'GoldenRod', 'Salmon', 'Tan', 'HoneyDew', 'HotPink', 'IndianRed',
    'Ivory', 'Khaki', 'Lavender', 'LavenderBlush', 'LawnGreen', 'LemonChiffon', 'LightBlue', 'LightCoral',
    'LightCyan', 'LightGoldenRodYellow', 'LightGray', 'LightGrey', 'LightGreen', 'LightPink', 'LightSalmon',
    'LightSeaGreen', 'LightSkyBlue', 'LightSlateGray', 'LightSlateGrey', 'LightSteelBlue', 'LightYellow', 'Lime',
    'LimeGreen', 'Linen', 'Magenta', 'MediumAquaMarine', 'MediumOrchid', 'MediumPurple', 'MediumSeaGreen',
    'MediumSlateBlue', 'MediumSpringGreen', 'MediumTurquoise', 'MediumVioletRed', 'MintCream', 'MistyRose',
    'Moccasin', 'NavajoWhite', 'OldLace', 'Olive', 'OliveDrab', 'Orange', 'OrangeRed', 'Orchid', 'PaleGoldenRod',
    'PaleGreen', 'PaleTurquoise', 'PaleVioletRed', 'PapayaWhip', 'PeachPuff', 'Peru', 'Pink', 'Plum', 'PowderBlue',
    'Purple', 'Red', 'RosyBrown', 'RoyalBlue', 'SaddleBrown', 'Green', 'SandyBrown', 'SeaGreen', 'SeaShell', 'Sienna',
    'Silver', 'SkyBlue', 'SlateBlue', 'SlateGray', 'SlateGrey', 'Snow', 'SpringGreen', 'SteelBlue', 'GreenYellow',
    'Teal', 'Thistle', 'Tomato', 'Turquoise', 'Violet', 'Wheat', 'White', 'WhiteSmoke', 'Yellow', 'YellowGreen']


def _font():
    try:
        return ImageFont.truetype('arial.ttf', 24)
    except IOError:
        return ImageFont.load_default()


def _text_size(font, s):
    left, top, right, bottom = font.getbbox(s)
    return right - left, bottom - top


def draw_bounding_box_on_image(image, ymin, xmin, ymax, xmax, color='red', thickness=4, display_str_list=(),
                               use_normalized_coordinates=True):
    """Box outline on a PIL image plus the display strings stacked above it (below when the box
    touches the top edge), black text on a `color` label background."""
    draw = ImageDraw.Draw(image)
    w, h = image.size
    if use_normalized_coordinates:
        left, right, top, bottom = xmin * w, xmax * w, ymin * h, ymax * h
    else:
        left, right, top, bottom = xmin, xmax, ymin, ymax
    draw.line([(left, top), (left, bottom), (right, bottom), (right, top), (left, top)], width=thickness, fill=color)
    font = _font()
    heights = [_text_size(font, s)[1] for s in display_str_list]
    total = (1 + 2 * 0.05) * sum(heights)
    text_bottom = top if top > total else bottom + total
    for s in display_str_list[::-1]:
        tw, th = _text_size(font, s)
        margin = np.ceil(0.05 * th)
        draw.rectangle([(left, text_bottom - th - 2 * margin), (left + tw, text_bottom)], fill=color)
        draw.text((left + margin, text_bottom - th - margin), s, fill='black', font=font)
        text_bottom -= th - 2 * margin


def draw_bounding_box_on_image_array(image, ymin, xmin, ymax, xmax, color='red', thickness=4, display_str_list=(),
                                     use_normalized_coordinates=True):
    """The same on a uint8 [H, W, 3] array, in place (returned too)."""
    pil = Image.fromarray(np.uint8(image)).convert('RGB')
    draw_bounding_box_on_image(pil, ymin, xmin, ymax, xmax, color, thickness, display_str_list,
                               use_normalized_coordinates)
    np.copyto(image, np.array(pil))
    return image


def draw_mask_on_image_array(image, mask, color='red', alpha=0.4):
    """Blend a 0/1 uint8 mask [H, W] into the uint8 image in `color` with opacity alpha."""
    if image.dtype != np.uint8:
        raise ValueError('`image` not of type np.uint8')
    if mask.dtype != np.uint8:
        raise ValueError('`mask` not of type np.uint8')
    if np.any((mask != 0) & (mask != 1)):
        raise ValueError('`mask` elements should be in [0, 1]')
    if image.shape[:2] != mask.shape:
        raise ValueError('The image has spatial dimensions %s but the mask has dimensions %s'
                         % (image.shape[:2], mask.shape))
    rgb = np.array(ImageColor.getrgb(color), np.float64)
    solid = Image.fromarray(np.uint8(np.ones(mask.shape + (1,)) * rgb)).convert('RGBA')
    alpha_img = Image.fromarray(np.uint8(255.0 * alpha * mask)).convert('L')
    out = Image.composite(solid, Image.fromarray(image), alpha_img)
    np.copyto(image, np.array(out.convert('RGB')))


def draw_keypoints_on_image(image, keypoints, color='red', radius=2, use_normalized_coordinates=True):
    """Filled circles at keypoints [K, 2] = (y, x) on a PIL image."""
    draw = ImageDraw.Draw(image)
    w, h = image.size
    for y, x in keypoints:
        if use_normalized_coordinates:
            x, y = w * x, h * y
        draw.ellipse([(x - radius, y - radius), (x + radius, y + radius)], outline=color, fill=color)


def draw_keypoints_on_image_array(image, keypoints, color='red', radius=2, use_normalized_coordinates=True):
    pil = Image.fromarray(np.uint8(image)).convert('RGB')
    draw_keypoints_on_image(pil, keypoints, color, radius, use_normalized_coordinates)
    np.copyto(image, np.array(pil))


def visualize_boxes_and_labels_on_image_array(image, boxes, classes, scores, category_index, instance_masks=None,
                                              instance_boundaries=None, keypoints=None,
                                              use_normalized_coordinates=True, max_boxes_to_draw=40,
                                              min_score_thresh=.2, agnostic_mode=False, line_thickness=3,
                                              groundtruth_box_visualization_color='red', skip_scores=False,
                                              skip_labels=False):
    """Overlay the boxes [N, 4] (ymin, xmin, ymax, xmax) whose score passes min_score_thresh
    (all when scores is None: ground truth, drawn in one colour), labelled 'name: NN%', one
    colour per class (STANDARD_COLORS[class % len]); boxes at the same location share one
    label block.  At most max_boxes_to_draw of the first boxes are considered.  In place."""
    display = collections.defaultdict(list)
    colour = collections.defaultdict(str)
    masks, bounds, kps = {}, {}, collections.defaultdict(list)
    n = boxes.shape[0] if not max_boxes_to_draw else min(max_boxes_to_draw, boxes.shape[0])
    for i in range(n):
        if scores is not None and not scores[i] > min_score_thresh:
            continue
        box = tuple(boxes[i].tolist())
        if instance_masks is not None:
            masks[box] = instance_masks[i]
        if instance_boundaries is not None:
            bounds[box] = instance_boundaries[i]
        if keypoints is not None:
            kps[box].extend(keypoints[i])
        if scores is None:
            colour[box] = groundtruth_box_visualization_color
            continue
        text = ''
        if not skip_labels and not agnostic_mode:
            name = category_index[classes[i]]['name'] if classes[i] in category_index else 'N/A'
            text = str(name)
        if not skip_scores:
            pct = '{}%'.format(int(100 * scores[i]))
            text = pct if not text else '{}: {}'.format(text, pct)
        display[box].append(text)
        colour[box] = 'DarkOrange' if agnostic_mode else STANDARD_COLORS[classes[i] % len(STANDARD_COLORS)]
    for box, c in colour.items():
        ymin, xmin, ymax, xmax = box
        if box in masks:
            draw_mask_on_image_array(image, masks[box], color=c)
        if box in bounds:
            draw_mask_on_image_array(image, bounds[box], color='red', alpha=1.0)
        draw_bounding_box_on_image_array(image, ymin, xmin, ymax, xmax, color=c, thickness=line_thickness,
                                         display_str_list=display[box],
                                         use_normalized_coordinates=use_normalized_coordinates)
        if box in kps:
            draw_keypoints_on_image_array(image, kps[box], color=c, radius=line_thickness / 2,
                                          use_normalized_coordinates=use_normalized_coordinates)
    return image
