"""Training data on device (reference yolox/data): the mosaic / mixup / affine / HSV / mirror
sample pipeline over dataset images resident in HBM.  This directory also holds the BN
calibration statistics (bn_stats_*.npz) the planner's synthetic weights use."""
from .mosaic import (AugParams, GpuMosaicDetection, MosaicBatches, ResidentImages, SyntheticDetectionDataset,
                     TrainTransform)

MosaicDetection = GpuMosaicDetection  # the reference's name (datasets/mosaicdetection.py:35)

__all__ = ["AugParams", "GpuMosaicDetection", "MosaicDetection", "MosaicBatches", "ResidentImages",
           "SyntheticDetectionDataset", "TrainTransform"]
