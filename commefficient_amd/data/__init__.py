from .fed_dataset import FedDataset, FedSampler
from .image_datasets import (ArrayImageFedDataset, FedCIFAR10, FedCIFAR100, FedEMNIST,
                             FedImageNet, SyntheticImageFedDataset, make_synthetic)

__all__ = ["FedDataset", "FedSampler", "ArrayImageFedDataset", "FedCIFAR10", "FedCIFAR100",
           "FedEMNIST", "FedImageNet", "SyntheticImageFedDataset", "make_synthetic"]
