from . import flow_viz  # noqa: F401
from .utils import InputPadder, forward_interpolate, bilinear_sampler, coords_grid, upflow8  # noqa: F401
