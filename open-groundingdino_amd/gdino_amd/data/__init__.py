"""ODVG data path: dataset, transforms, collate and
DataLoader-side text preprocessing."""
from .odvg import ODVGCollator, ODVGDataset, TextPreprocessor, build_odvg, collate_fn  # noqa: F401
from .transforms import make_transforms  # noqa: F401
