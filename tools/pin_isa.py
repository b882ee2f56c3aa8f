"""Re-pin the bench kernels' instruction streams (tests/golden/kernel_isa.json) after a deliberate
kernel change:  python tools/pin_isa.py   (what tests/test_kernel_resources.py compares against)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "polar-code-pytorch-sionna_amd"), os.path.join(ROOT, "tests")]
import test_kernel_resources as t  # noqa: E402
from polar_amd import build  # noqa: E402

pins = t.current_pins()
pins["source_hash"] = build.source_hash()
json.dump(pins, open(t.PIN_PATH, "w"), indent=1, sort_keys=True)
print(json.dumps(pins, indent=1))
