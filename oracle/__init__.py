"""CPU oracle for itzmeanjan/rlnc 0.8.5 — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package.
The product (rlnc_amd / librlnc_hip.so) never touches it.  See rlnc_oracle.h for the parity status.
"""
from .oracle import Oracle, OracleDecoder, load  # noqa: F401
