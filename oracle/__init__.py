"""TEST INFRASTRUCTURE ONLY: Python loader for the CPU oracle (fa_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package.  See fa_oracle.h for what the oracle restates and how it
is pinned.
"""
from .fa_oracle import (  # noqa: F401
    ORACLE_LIB,
    attention,
    attention_heads,
    attention_rows,
    build,
    f16_bits_to_f32,
    gen_inputs,
    load,
    max_abs_diff,
)
