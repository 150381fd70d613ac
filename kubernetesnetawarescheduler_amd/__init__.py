"""MI355X-native network-aware pod placement engine.

Drop-in for the placement decision of pablojara/kubernetesNetAwareScheduler
(scheduler/scheduler.go:239-394): hand-written gfx950 HIP kernels behind the
C ABI of include/nas.h (libnas.so, built in-tree).  This Python package is
plumbing for tests and benchmarks; the host mirror of the reference's
CustomScheduler lives in host/ (C++).
"""
from ._lib import (K_CANDIDATES, NAS_DT_BF16, NAS_DT_I8, NAS_EMPTY, NAS_NONE, NasError,  # noqa: F401
                   LIB_PATH)
from .engine import FIELDS, Engine, LocalGroup, local_ranks  # noqa: F401
