"""API object models: builders for Pods, Nodes, PodGroups, ElasticQuotas,
NodeResourceTopologies, PDBs, PriorityClasses, and the MI355X node model."""
from .mi355x import (GPU, GPU_MEMORY, GPU_XCD, INDEX_ANNOTATION, PARTITION_ANNOTATION, PARTITION_LABEL,
                     TOPOLOGY_ANNOTATION, GpuInfo, default_gpus, mi355x_node, mi355x_nrt)
from .objects import (POD_GROUP_LABEL, make_container, make_elastic_quota, make_node, make_nrt, make_pdb, make_pod,
                      make_pod_group, make_priority_class, nrt_zone)

__all__ = [
    "GPU", "GPU_MEMORY", "GPU_XCD", "INDEX_ANNOTATION", "PARTITION_ANNOTATION", "PARTITION_LABEL",
    "TOPOLOGY_ANNOTATION", "GpuInfo", "default_gpus", "mi355x_node", "mi355x_nrt", "POD_GROUP_LABEL",
    "make_container", "make_elastic_quota", "make_node", "make_nrt", "make_pdb", "make_pod", "make_pod_group",
    "make_priority_class", "nrt_zone",
]
