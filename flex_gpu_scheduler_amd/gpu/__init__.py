"""GPU side of the control plane: MI355X discovery (sysfs/KFD) and load
telemetry; HIP device probes live in ops/hip_probe.py."""
from .discovery import GpuDevice, HostInfo, discover_gpus, discover_host, fake_host  # noqa: F401
from .telemetry import HostSampler, LoadWatcherService, NodeTelemetry, WatcherFetcher  # noqa: F401
