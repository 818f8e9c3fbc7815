"""Kubelet device-plugin API v1beta1 (k8s.io/kubelet/pkg/apis/deviceplugin/
v1beta1/api.proto), built at import time from descriptors.

The image has grpcio and protobuf but no protoc/grpc_tools, so the message
types are declared here field-by-field (names, numbers and types match the
upstream .proto, which is what wire compatibility depends on) and turned into
classes with protobuf's message factory. The gRPC method paths are the
upstream ones (`/v1beta1.Registration/Register`, `/v1beta1.DevicePlugin/...`).
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "v1beta1"
VERSION = "v1beta1"
KUBELET_SOCKET = "kubelet.sock"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins/"
HEALTHY, UNHEALTHY = "Healthy", "Unhealthy"

_F = descriptor_pb2.FieldDescriptorProto
_STR, _BOOL, _I64, _I32, _MSG = _F.TYPE_STRING, _F.TYPE_BOOL, _F.TYPE_INT64, _F.TYPE_INT32, _F.TYPE_MESSAGE
_OPT, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED

# name -> [(field, number, type, label, message type name)]
_MESSAGES: dict[str, list[tuple]] = {
    "DevicePluginOptions": [("pre_start_required", 1, _BOOL, _OPT, None),
                            ("get_preferred_allocation_available", 2, _BOOL, _OPT, None)],
    "RegisterRequest": [("version", 1, _STR, _OPT, None), ("endpoint", 2, _STR, _OPT, None),
                        ("resource_name", 3, _STR, _OPT, None), ("options", 4, _MSG, _OPT, "DevicePluginOptions")],
    "Empty": [],
    "ListAndWatchResponse": [("devices", 1, _MSG, _REP, "Device")],
    "TopologyInfo": [("nodes", 1, _MSG, _REP, "NUMANode")],
    "NUMANode": [("ID", 1, _I64, _OPT, None)],
    "Device": [("ID", 1, _STR, _OPT, None), ("health", 2, _STR, _OPT, None), ("topology", 3, _MSG, _OPT, "TopologyInfo")],
    "PreStartContainerRequest": [("devicesIDs", 1, _STR, _REP, None)],
    "PreStartContainerResponse": [],
    "PreferredAllocationRequest": [("container_requests", 1, _MSG, _REP, "ContainerPreferredAllocationRequest")],
    "ContainerPreferredAllocationRequest": [("available_deviceIDs", 1, _STR, _REP, None),
                                            ("must_include_deviceIDs", 2, _STR, _REP, None),
                                            ("allocation_size", 3, _I32, _OPT, None)],
    "PreferredAllocationResponse": [("container_responses", 1, _MSG, _REP, "ContainerPreferredAllocationResponse")],
    "ContainerPreferredAllocationResponse": [("deviceIDs", 1, _STR, _REP, None)],
    "AllocateRequest": [("container_requests", 1, _MSG, _REP, "ContainerAllocateRequest")],
    "ContainerAllocateRequest": [("devicesIDs", 1, _STR, _REP, None)],
    "AllocateResponse": [("container_responses", 1, _MSG, _REP, "ContainerAllocateResponse")],
    "ContainerAllocateResponse": [("envs", 1, _MSG, _REP, "ContainerAllocateResponse.EnvsEntry"),
                                  ("mounts", 2, _MSG, _REP, "Mount"), ("devices", 3, _MSG, _REP, "DeviceSpec"),
                                  ("annotations", 4, _MSG, _REP, "ContainerAllocateResponse.AnnotationsEntry")],
    "Mount": [("container_path", 1, _STR, _OPT, None), ("host_path", 2, _STR, _OPT, None),
              ("read_only", 3, _BOOL, _OPT, None)],
    "DeviceSpec": [("container_path", 1, _STR, _OPT, None), ("host_path", 2, _STR, _OPT, None),
                   ("permissions", 3, _STR, _OPT, None)],
}
_MAP_ENTRIES = {"ContainerAllocateResponse": ["EnvsEntry", "AnnotationsEntry"]}

SERVICES = {
    "Registration": {"Register": ("RegisterRequest", "Empty", False)},
    "DevicePlugin": {
        "GetDevicePluginOptions": ("Empty", "DevicePluginOptions", False),
        "ListAndWatch": ("Empty", "ListAndWatchResponse", True),
        "GetPreferredAllocation": ("PreferredAllocationRequest", "PreferredAllocationResponse", False),
        "Allocate": ("AllocateRequest", "AllocateResponse", False),
        "PreStartContainer": ("PreStartContainerRequest", "PreStartContainerResponse", False),
    },
}


def _build():
    fdp = descriptor_pb2.FileDescriptorProto(name="deviceplugin_v1beta1.proto", package=PACKAGE, syntax="proto3")
    for name, fields in _MESSAGES.items():
        m = fdp.message_type.add(name=name)
        for entry in _MAP_ENTRIES.get(name, []):
            e = m.nested_type.add(name=entry)
            e.options.map_entry = True
            e.field.add(name="key", number=1, type=_STR, label=_OPT)
            e.field.add(name="value", number=2, type=_STR, label=_OPT)
        for fname, num, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = f".{PACKAGE}.{tname}"
    for sname, methods in SERVICES.items():
        s = fdp.service.add(name=sname)
        for mname, (req, resp, stream) in methods.items():
            s.method.add(name=mname, input_type=f".{PACKAGE}.{req}", output_type=f".{PACKAGE}.{resp}",
                         server_streaming=stream)
    pool = descriptor_pool.DescriptorPool()
    fd = pool.Add(fdp)
    fd = pool.FindFileByName(fdp.name)
    return {name: message_factory.GetMessageClass(fd.message_types_by_name[name]) for name in _MESSAGES}


pb = type("pb", (), _build())


def method_path(service: str, method: str) -> str:
    return f"/{PACKAGE}.{service}/{method}"
