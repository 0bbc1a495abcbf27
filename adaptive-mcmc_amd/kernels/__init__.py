"""Import surface of the reference (python/kernels/__init__.py:1):
`from kernels import ARWMH, ARWMHState, ARWMHAdaptState`.

`from kernels import ASSS, ASSSState, ASSSAdaptState` as the reference's
python/kernels/asss.py.  NUMPYRO NUTS / SA wrappers are outside the
accelerated path."""
from .arwmh import ARWMH, ARWMHAdaptState, ARWMHState, init_to_uniform, pack_scale, packed_size, unpack_scale
from .asss import ASSS, ASSSAdaptState, ASSSState
from .pooled import PooledAdaptState, PooledARWMH, PooledState
from .random import PRNGKey, split

__all__ = ["ARWMH", "ARWMHState", "ARWMHAdaptState", "init_to_uniform", "pack_scale", "unpack_scale",
           "packed_size", "PRNGKey", "split", "PooledARWMH", "PooledState", "PooledAdaptState",
           "ASSS", "ASSSState", "ASSSAdaptState"]
