"""Negative control (GPU) for the allocator-churn regression tests (tests/test_gpu_train.py, tests/test_gpu_churn.py):
the same tests with hiseg._lib.Desc's holding undone -- descriptor pointer fields store bare addresses again, as
before round 4, and nothing else keeps fg_gate's Dropout2d mask alive between the forward and the backward (the
round-3 flake).  The churn tests should then FAIL; with the holding in place they pass (developer tool).

Usage: python tools/churn_control.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "human-instance-segmentation_amd"), os.path.join(ROOT, "tests", "golden"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from hiseg import _lib as L  # noqa: E402
import test_gpu_churn  # noqa: E402
import test_gpu_train  # noqa: E402


def bare_address(self, name, value):
    """Desc.__setattr__ without the hold: the pre-round-4 behaviour (only the address is kept)."""
    if name in self._ptr_fields and value is not None and not isinstance(value, int):
        value = (value if isinstance(value, torch.Tensor) else value.t).data_ptr()
    ctypes.Structure.__setattr__(self, name, value)


def run(label, fn):
    try:
        fn()
        print(f"{label}: test PASSED")
        return True
    except AssertionError as e:
        print(f"{label}: test FAILED ({str(e).splitlines()[0][:160] if str(e) else 'assertion'})")
        return False


TESTS = [("B0 step", test_gpu_train.test_train_step_independent_of_allocator_churn_between_forward_and_backward),
         ("C3 step", test_gpu_churn.test_c3_train_step_independent_of_allocator_churn),
         ("C5 distillation step", test_gpu_churn.test_c5_distillation_step_independent_of_allocator_churn)]
ok_with = {name: run(f"{name}, with the holds (product)", fn) for name, fn in TESTS}
L.STRICT_PTRS = False
L.Desc.__setattr__ = bare_address
ok_without = {name: run(f"{name}, control: holds undone", fn) for name, fn in TESTS}
for name, _ in TESTS:
    if ok_with[name] and not ok_without[name]:
        print(f"control {name}: the churn test catches a released buffer without the holds and passes with them")
    elif ok_with[name]:
        print(f"control {name}: the churn test passes without the holds too (nothing it exercises depends on them)")
    else:
        print(f"control {name}: the churn test FAILS with the holds in place")
