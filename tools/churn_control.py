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

from hiseg import _lib as L  # noqa: E402
import test_gpu_train  # noqa: E402


def bare_address(self, name, value):
    """Desc.__setattr__ without the hold: the pre-round-4 behaviour (only the address is kept)."""
    if name in self._ptr_fields and value is not None and not isinstance(value, int):
        value = getattr(value, "t", value).data_ptr()
    ctypes.Structure.__setattr__(self, name, value)


def run(label, fn):
    try:
        fn()
        print(f"{label}: test PASSED")
        return True
    except AssertionError as e:
        print(f"{label}: test FAILED ({str(e).splitlines()[0][:160] if str(e) else 'assertion'})")
        return False


ok_with = run("with the holds (product)", test_gpu_train.test_train_step_independent_of_allocator_churn_between_forward_and_backward)
L.STRICT_PTRS = False
L.Desc.__setattr__ = bare_address
ok_without = run("control, holds undone", test_gpu_train.test_train_step_independent_of_allocator_churn_between_forward_and_backward)
if ok_with and not ok_without:
    print("control: the churn test catches the released-mask bug and passes with the fix")
elif ok_with:
    print("control: the churn test did NOT catch the bug (passes without the holds)")
else:
    print("control: the churn test fails with the holds in place")
