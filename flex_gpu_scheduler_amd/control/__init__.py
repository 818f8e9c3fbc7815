"""Python control plane: HTTP API server, clients, informers, controllers,
leader election, the remote-mode scheduler bridge, node agent and telemetry.

None of this is on the per-pod scheduling hot path — that stays in the C++
core; the control plane moves objects in and out of the native store."""
from .apiserver import ApiServer  # noqa: F401
from .client import ApiException, Client, LocalClient, RestClient, client_for  # noqa: F401
from .controllers import ControllerManager, ElasticQuotaController, PodGroupController  # noqa: F401
from .informer import Informer, InformerFactory, WorkQueue  # noqa: F401
from .leaderelection import LeaderElector  # noqa: F401
