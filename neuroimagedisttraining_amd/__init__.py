"""neuroimagedisttraining_amd — an MI355X-native federated-learning simulator for neuroimaging.

Capabilities mirror bishalth01/NeuroImageDistTraining (FedML-derived): FedAvg, SalientGrads
(SNIP-saliency global sparse masks), DisPFL, SubAvg, Ditto, D-PSGD, FedFomo, Local, plus
FedProx and Krum/median/trimmed-mean robust aggregation.  The hot path is a client-batched
executor (many virtual clients per GPU in lockstep) built on hand-written CDNA4 HIP kernels
(`csrc/kernels/*.hip`, loaded through :mod:`neuroimagedisttraining_amd.ops`) with
RCCL (``torch.distributed`` backend ``"nccl"``) aggregation over xGMI, one process per GPU.

Subpackages
-----------
core        trainer ABC, partitioners, robust aggregation, message/comm API, topology
models      AlexNet3D family, 3D ResNets, 2D CNN zoo, logistic regression
data        synthetic ABCD-shape volumes, tabular non-IID data, dataset loaders
algorithms  standalone FL algorithms (reference-semantics, torch eager)
engine      client-batched executor (HIP kernels, stacked per-client weights)
ops         Python bindings of the HIP kernels
parallel    process-per-GPU runtime, client sharding, bucketed RCCL collectives
utils       FLOP counting, logging, timers, checkpoint/resume
"""

__version__ = "0.1.0"
