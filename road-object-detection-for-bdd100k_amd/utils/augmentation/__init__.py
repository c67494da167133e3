"""Training-time augmentation (reference utils/augmentation/): parameter sampling on the host,
image and box transforms in librod (rod_augment_images / rod_augment_boxes)."""
