"""Reference ``fedml_api/model/cv/test_cnn.py``: print the complexity of ``CNN_DropOut`` on a 1x28x28 input.

The reference uses ``ptflops`` (not installed); this uses the framework's own hook-based counter
(``neuroimagedisttraining_amd.utils.flops``, which also counts Conv3d)."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..")))

from fedml_api.model.cv.cnn import CNN_DropOut  # noqa: E402
from neuroimagedisttraining_amd.utils.flops import count_model_param_flops  # noqa: E402


def complexity(net, input_shape=(1, 28, 28)):
    flops = count_model_param_flops(net, full=True, input_shape=input_shape)
    params = sum(p.numel() for p in net.parameters())
    return flops, params


if __name__ == "__main__":
    net = CNN_DropOut()
    flops, params = complexity(net)
    print(params)
    print('{:<30}  {:<8}'.format('Computational complexity: ', "%.2f MMac" % (flops / 2e6)))
    print('{:<30}  {:<8}'.format('Number of parameters: ', "%.2f k" % (params / 1e3)))
