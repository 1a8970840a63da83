"""plaincv_amd -- MI355X-native training hot path for GeorgTirp/plainCV.

Import order matters: torch is imported before libplaincv_hip.so is loaded so
the process shares torch's HIP runtime (both bind the soname libamdhip64.so.7).
"""
import torch  # noqa: F401

__version__ = "0.1.0"
