from .ddp import DistInfo, init_distributed, wrap_model, all_reduce_mean, barrier, cleanup, spawn  # noqa: F401
