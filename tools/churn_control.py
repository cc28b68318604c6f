"""Negative control (GPU) for test_train_step_independent_of_allocator_churn_between_forward_and_backward: the same
test with dropout_mask's keep-alive undone (the pre-fix behaviour) -- the test should then fail (developer tool)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "human-instance-segmentation_amd"), os.path.join(ROOT, "tests", "golden"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

from hiseg import train_engine as TE  # noqa: E402
import test_gpu_train  # noqa: E402

orig = TE.dropout_mask


def unkept(T, m, N, C, device):
    out = orig(T, m, N, C, device)
    if out is not None:
        T.keep.pop()
    return out


TE.dropout_mask = unkept
try:
    test_gpu_train.test_train_step_independent_of_allocator_churn_between_forward_and_backward()
    print("control: test PASSED without the keep-alive (the test does not catch the bug)")
except AssertionError:
    print("control: test FAILED without the keep-alive, as it should")
