from . import frame_utils  # noqa: F401
from .synthetic import synthetic_batch, SyntheticFlowDataset  # noqa: F401
