"""Import surface of the reference's `kernels` package (python/kernels/__init__.py:1-2).

The reference's own package keeps its name; a maintainer swaps its first two
lines for

    from kernels_amd import ARWMH, ARWMHState, ARWMHAdaptState
    from kernels_amd import ASSS, ASSSState, ASSSAdaptState

and leaves line 3 (`from .numpyro_kernels import NUTS, HMCState, SA, SAState`)
alone: the NumPyro NUTS / SA wrappers are outside the accelerated path
(SURVEY.md §2), and this package is named `kernels_amd` precisely so that it
does not shadow them (tests/test_integration.py)."""
from .arwmh import ARWMH, ARWMHAdaptState, ARWMHState, init_to_uniform, pack_scale, packed_size, unpack_scale
from .asss import ASSS, ASSSAdaptState, ASSSState
from .pooled import PooledAdaptState, PooledARWMH, PooledState
from .random import PRNGKey, split
from .checkpoint import load_state, load_state_dict, save_state, state_dict

__all__ = ["ARWMH", "ARWMHState", "ARWMHAdaptState", "init_to_uniform", "pack_scale", "unpack_scale",
           "packed_size", "PRNGKey", "split", "PooledARWMH", "PooledState", "PooledAdaptState",
           "ASSS", "ASSSState", "ASSSAdaptState", "state_dict", "load_state_dict", "save_state", "load_state"]
