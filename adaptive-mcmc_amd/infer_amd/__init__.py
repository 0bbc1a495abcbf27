"""Driver surface around the kernels: `infer.MCMC` (numpyro's MCMC as the
reference scripts use it) and numpyro-style diagnostics."""
from . import diagnostics
from .diagnostics import (autocorrelation, autocovariance, effective_sample_size, gelman_rubin, hpdi,
                          print_summary, split_gelman_rubin, summary)
from .mcmc import MCMC

__all__ = ["MCMC", "diagnostics", "autocorrelation", "autocovariance", "effective_sample_size", "gelman_rubin",
           "split_gelman_rubin", "hpdi", "summary", "print_summary"]
