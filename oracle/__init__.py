"""CPU oracle for the placement path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package.  The product (kubernetesnetawarescheduler_amd) never
does; see oracle.c's header for what each function restates (reference
file:line) and how parity is pinned.
"""
from .oracle import *  # noqa: F401,F403
