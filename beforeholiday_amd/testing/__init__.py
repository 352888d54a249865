from .common_utils import HAS_GPU, SKIP_FLAKY_TEST, TEST_WITH_ROCM, skipFlakyTest, skipIfNoGPU, skipIfRocm
