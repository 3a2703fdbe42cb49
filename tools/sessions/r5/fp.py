"""Print the convergence test's cohort fingerprint (to record it next to the fp32 trajectory)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import test_gpu_convergence as T  # noqa: E402

vol, labels, splits = T._cohort()
print("FINGERPRINT", T._fingerprint(vol, labels, splits))
