"""flex_gpu_scheduler_amd — an MI355X-native Kubernetes scheduler-plugin suite.

Capabilities of WLBF/flex-gpu-scheduler (scheduler-plugins fork + FlexGPU),
rebuilt MI355X-first: a C++ scheduling core (framework runtime, queue, cache,
preemption, plugins) with a Python control plane (config, store/HTTP API,
controllers, node agent, telemetry) and HIP/RCCL probes for the GPU side.
"""
__version__ = "0.1.0"

from .config import ConfigError, SchedulerConfiguration, load_config  # noqa: F401
from .scheduler import FakeClock, Store, new_scheduler  # noqa: F401
