"""Build A/B variants of liblgm_amd.so: python scripts/ab_variants.py NAME:DEF1,DEF2 NAME2:..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lgm_amd import build as B  # noqa: E402

for spec in sys.argv[1:]:
    name, _, defs = spec.partition(":")
    out = os.path.join(B.HERE, "_lib", "variants", f"lib_{name}.so")
    B.build(out=out, defines=[d for d in defs.split(",") if d])
    print(out)
