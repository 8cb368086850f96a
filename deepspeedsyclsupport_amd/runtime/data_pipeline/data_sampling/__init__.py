from .data_sampler import DeepSpeedDataSampler
from .data_analyzer import DataAnalyzer
from .indexed_dataset import MMapIndexedDataset, MMapIndexedDatasetBuilder, make_builder, make_dataset
