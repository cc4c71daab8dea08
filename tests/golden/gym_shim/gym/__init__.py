"""Minimal stand-in for gym==0.17.2 (not installable offline), used ONLY by gen_golden.py to
instantiate the reference LoadBalanceEnv in this container.  Our own scaffolding, not reference
code: just the two space classes and the Env base the reference touches (env.py:20-26,163-182)."""
from . import spaces  # noqa: F401


class Env:
    metadata = {}
