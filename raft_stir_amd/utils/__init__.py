from .padder import InputPadder
from .geometry import coords_grid, bilinear_sampler, upflow8, forward_interpolate

__all__ = ["InputPadder", "coords_grid", "bilinear_sampler", "upflow8", "forward_interpolate"]
