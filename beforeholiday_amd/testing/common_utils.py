"""Test helpers (reference: apex/testing/common_utils.py:12-33)."""
import os
import unittest

import torch

TEST_WITH_ROCM = os.getenv("APEX_TEST_WITH_ROCM", "0") == "1" or torch.version.hip is not None
SKIP_FLAKY_TEST = os.getenv("APEX_SKIP_FLAKY_TEST", "0") == "1"
HAS_GPU = torch.cuda.is_available()


def skipIfRocm(fn):
    return unittest.skipIf(TEST_WITH_ROCM, "test doesn't currently work on the ROCm stack")(fn)


def skipFlakyTest(fn):
    return unittest.skipIf(SKIP_FLAKY_TEST, "Test is flaky.")(fn)


def skipIfNoGPU(fn):
    return unittest.skipIf(not HAS_GPU, "needs a GPU")(fn)
