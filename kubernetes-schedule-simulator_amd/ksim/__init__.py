"""ksim — MI355X-native per-pod scheduling cycle of the kube-scheduler v1.10 path driven by
xiaoxubeii/kubernetes-schedule-simulator.  The compute path is libksim.so (HIP, gfx950);
this package is the host-side mirror of the reference's plugin/simulator interface."""
from . import abi, ingest, labels, quantity, scheduler  # noqa: F401
from .abi import KsimError, KsimUnsupported  # noqa: F401
from .ingest import Cluster  # noqa: F401
from .scheduler import ClusterCapacity, GenericScheduler, expand_simulation_pods, fit_error_message, provider  # noqa: F401
