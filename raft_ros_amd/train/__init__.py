from .loss import sequence_loss, metrics_to_host, MAX_FLOW  # noqa: F401
from .optim import fetch_optimizer, count_parameters  # noqa: F401
