"""BDD100K label JSON -> Pascal-VOC XML (reference convert/json2xml/{bdd2voc,parseJson,
pascal_voc_io}.py): one XML per frame that has at least one object of the kept categories,
boxes as int(x1), int(y1), int(x2), int(y2), image size 720x1280x3, no lxml (the standard
library's ElementTree + minidom for the indentation).

  python convert/bdd2voc.py --json_dir <labels/100k/train> --save_dir <Annotations>
"""
import argparse
import json
import os
from xml.dom import minidom
from xml.etree.ElementTree import Element, SubElement, tostring

# parseJson.py:8-10 — the converter keeps only these categories (so classes 5 / 7 / 9 of
# dataset/bdd100k.py never get ground truth)
CATEGORIES = ['bus', 'traffic light', 'traffic sign', 'person', 'truck', 'car', 'rider']


def parse_json(json_file, categories=CATEGORIES):
    """[[x1, y1, x2, y2, category], ...] of the first frame's objects in `categories`."""
    with open(json_file) as f:
        info = json.load(f)
    objs = []
    for o in info['frames'][0]['objects']:
        if o['category'] in categories:
            b = o['box2d']
            objs.append([int(b['x1']), int(b['y1']), int(b['x2']), int(b['y2']), o['category']])
    return objs


def voc_xml(filename, objs, img_size=(720, 1280, 3), database='BDD100K', path=None):
    """The annotation tree PascalVocWriter writes (pascal_voc_io.py:25-89): folder, filename.jpg,
    path, source/database, size (width, height, depth), segmented 0, one object per box with
    pose Unspecified, truncated 0, difficult 0 and the bndbox corners."""
    top = Element('annotation')
    SubElement(top, 'folder').text = 'BDD100K'
    SubElement(top, 'filename').text = filename + '.jpg'
    SubElement(top, 'path').text = path
    SubElement(SubElement(top, 'source'), 'database').text = database
    size = SubElement(top, 'size')
    SubElement(size, 'width').text = str(img_size[1])
    SubElement(size, 'height').text = str(img_size[0])
    SubElement(size, 'depth').text = str(img_size[2]) if len(img_size) == 3 else '1'
    SubElement(top, 'segmented').text = '0'
    for xmin, ymin, xmax, ymax, name in objs:
        ob = SubElement(top, 'object')
        SubElement(ob, 'name').text = str(name)
        SubElement(ob, 'pose').text = 'Unspecified'
        SubElement(ob, 'truncated').text = '0'
        SubElement(ob, 'difficult').text = '0'
        bb = SubElement(ob, 'bndbox')
        for k, v in (('xmin', xmin), ('ymin', ymin), ('xmax', xmax), ('ymax', ymax)):
            SubElement(bb, k).text = str(v)
    return top


def write_voc(save_dir, filename, objs, img_size=(720, 1280, 3)):
    xml = minidom.parseString(tostring(voc_xml(filename, objs, img_size), 'utf-8')).toprettyxml(indent='  ')
    with open(os.path.join(save_dir, filename + '.xml'), 'w') as f:
        f.write(xml)


def convert_dir(json_dir, save_dir, img_size=(720, 1280, 3)):
    """bdd2voc.py:7-29: walk json_dir, one XML per JSON with kept objects; returns (written, skipped)."""
    os.makedirs(save_dir, exist_ok=True)
    written, skipped = 0, []
    for dirpath, _, names in os.walk(json_dir):
        for name in sorted(names):
            if not name.endswith('.json'):
                continue
            objs = parse_json(os.path.join(dirpath, name))
            if objs:
                write_voc(save_dir, name[:-5], objs, img_size)
                written += 1
            else:
                skipped.append(name)
    return written, skipped


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument('--json_dir', required=True)
    ap.add_argument('--save_dir', default='../Annotations')
    a = ap.parse_args(argv)
    n, skipped = convert_dir(a.json_dir, a.save_dir)
    print('wrote %d annotation files; %d frames without kept objects' % (n, len(skipped)))


if __name__ == '__main__':
    main()
