"""Convert a VOC-layout dataset (BDD100K after convert/bdd2voc.py) to TFRecords
(reference tf_convert_data.py; same flags and defaults, no TensorFlow):

  python tf_convert_data.py --dataset_name=bdd100k --dataset_dir=<dir with Annotations/ JPEGImages/> \
      --output_name=bdd100k_train --output_dir=./dataset/bdd100k_TfRecord
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from dataset import pascalvoc_to_tfrecords  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument('--dataset_name', default='bdd100k')
    ap.add_argument('--dataset_dir', default='h:/Data/BDD100K/bdd/images/100k/')
    ap.add_argument('--output_name', default='bdd100k_val')
    ap.add_argument('--output_dir', default='./dataset/bdd100k_TfRecord')
    F = ap.parse_args(argv)
    if not F.dataset_dir:
        raise ValueError('You must supply the dataset directory with --dataset_dir')
    print('Dataset directory:', F.dataset_dir)
    print('Output directory:', F.output_dir)
    if F.dataset_name not in ('pascalvoc', 'bdd100k'):
        raise ValueError('Dataset [%s] was not recognized.' % F.dataset_name)
    return pascalvoc_to_tfrecords.run(F.dataset_dir, F.output_dir, F.output_name)


if __name__ == '__main__':
    main()
