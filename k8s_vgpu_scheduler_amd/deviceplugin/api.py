"""Kubelet DevicePlugin API v1beta1, built without protoc.

The image has grpcio + protobuf but no grpc_tools/protoc, so
the messages of k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto are
declared here as a FileDescriptorProto and materialised with the protobuf
runtime; the two services are wired with grpc generic handlers.  Field
numbers and names follow api.proto exactly (wire compatible with kubelet).
"""

from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "v1beta1"
VERSION = "v1beta1"
KUBELET_SOCKET = "/var/lib/kubelet/device-plugins/kubelet.sock"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins/"
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"

F = descriptor_pb2.FieldDescriptorProto
_STR, _BOOL, _I64, _I32, _MSG = F.TYPE_STRING, F.TYPE_BOOL, F.TYPE_INT64, F.TYPE_INT32, F.TYPE_MESSAGE
_OPT, _REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED

# name -> [(field, number, type, label, type_name)]
_MESSAGES = {
    "DevicePluginOptions": [("pre_start_required", 1, _BOOL, _OPT, None),
                            ("get_preferred_allocation_available", 2, _BOOL, _OPT, None)],
    "RegisterRequest": [("version", 1, _STR, _OPT, None), ("endpoint", 2, _STR, _OPT, None),
                        ("resource_name", 3, _STR, _OPT, None),
                        ("options", 4, _MSG, _OPT, "DevicePluginOptions")],
    "Empty": [],
    "ListAndWatchResponse": [("devices", 1, _MSG, _REP, "Device")],
    "TopologyInfo": [("nodes", 1, _MSG, _REP, "NUMANode")],
    "NUMANode": [("ID", 1, _I64, _OPT, None)],
    "Device": [("ID", 1, _STR, _OPT, None), ("health", 2, _STR, _OPT, None),
               ("topology", 3, _MSG, _OPT, "TopologyInfo")],
    "PreStartContainerRequest": [("devices_ids", 1, _STR, _REP, None)],
    "PreStartContainerResponse": [],
    "PreferredAllocationRequest": [("container_requests", 1, _MSG, _REP, "ContainerPreferredAllocationRequest")],
    "ContainerPreferredAllocationRequest": [("available_deviceIDs", 1, _STR, _REP, None),
                                            ("must_include_deviceIDs", 2, _STR, _REP, None),
                                            ("allocation_size", 3, _I32, _OPT, None)],
    "PreferredAllocationResponse": [("container_responses", 1, _MSG, _REP, "ContainerPreferredAllocationResponse")],
    "ContainerPreferredAllocationResponse": [("deviceIDs", 1, _STR, _REP, None)],
    "AllocateRequest": [("container_requests", 1, _MSG, _REP, "ContainerAllocateRequest")],
    "ContainerAllocateRequest": [("devices_ids", 1, _STR, _REP, None)],
    "AllocateResponse": [("container_responses", 1, _MSG, _REP, "ContainerAllocateResponse")],
    "CDIDevice": [("name", 1, _STR, _OPT, None)],
    "Mount": [("container_path", 1, _STR, _OPT, None), ("host_path", 2, _STR, _OPT, None),
              ("read_only", 3, _BOOL, _OPT, None)],
    "DeviceSpec": [("container_path", 1, _STR, _OPT, None), ("host_path", 2, _STR, _OPT, None),
                   ("permissions", 3, _STR, _OPT, None)],
}
# ContainerAllocateResponse has two map<string,string> fields (nested map entries).
_CAR = "ContainerAllocateResponse"


def _build():
    fdp = descriptor_pb2.FileDescriptorProto(name="mivgpu/deviceplugin/v1beta1/api.proto", package=PACKAGE,
                                             syntax="proto3")
    for mname, fields in _MESSAGES.items():
        m = fdp.message_type.add(name=mname)
        for fname, num, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = f".{PACKAGE}.{tname}"
    car = fdp.message_type.add(name=_CAR)
    for entry, num in (("EnvsEntry", 1), ("AnnotationsEntry", 4)):
        e = car.nested_type.add(name=entry)
        e.field.add(name="key", number=1, type=_STR, label=_OPT)
        e.field.add(name="value", number=2, type=_STR, label=_OPT)
        e.options.map_entry = True
        car.field.add(name="envs" if num == 1 else "annotations", number=num, type=_MSG, label=_REP,
                      type_name=f".{PACKAGE}.{_CAR}.{entry}")
    car.field.add(name="mounts", number=2, type=_MSG, label=_REP, type_name=f".{PACKAGE}.Mount")
    car.field.add(name="devices", number=3, type=_MSG, label=_REP, type_name=f".{PACKAGE}.DeviceSpec")
    car.field.add(name="cdi_devices", number=5, type=_MSG, label=_REP, type_name=f".{PACKAGE}.CDIDevice")
    pool = descriptor_pool.DescriptorPool()
    fd = pool.Add(fdp)
    classes = {}
    for name in list(_MESSAGES) + [_CAR]:
        desc = pool.FindMessageTypeByName(f"{PACKAGE}.{name}")
        classes[name] = message_factory.GetMessageClass(desc)
    return fd, classes


_FD, M = _build()

DevicePluginOptions = M["DevicePluginOptions"]
RegisterRequest = M["RegisterRequest"]
Empty = M["Empty"]
ListAndWatchResponse = M["ListAndWatchResponse"]
TopologyInfo = M["TopologyInfo"]
NUMANode = M["NUMANode"]
Device = M["Device"]
PreStartContainerRequest = M["PreStartContainerRequest"]
PreStartContainerResponse = M["PreStartContainerResponse"]
PreferredAllocationRequest = M["PreferredAllocationRequest"]
ContainerPreferredAllocationRequest = M["ContainerPreferredAllocationRequest"]
PreferredAllocationResponse = M["PreferredAllocationResponse"]
ContainerPreferredAllocationResponse = M["ContainerPreferredAllocationResponse"]
AllocateRequest = M["AllocateRequest"]
ContainerAllocateRequest = M["ContainerAllocateRequest"]
AllocateResponse = M["AllocateResponse"]
ContainerAllocateResponse = M[_CAR]
Mount = M["Mount"]
DeviceSpec = M["DeviceSpec"]
CDIDevice = M["CDIDevice"]

# (method, request class, response class, streaming response)
DEVICE_PLUGIN_METHODS = {
    "GetDevicePluginOptions": (Empty, DevicePluginOptions, False),
    "ListAndWatch": (Empty, ListAndWatchResponse, True),
    "GetPreferredAllocation": (PreferredAllocationRequest, PreferredAllocationResponse, False),
    "Allocate": (AllocateRequest, AllocateResponse, False),
    "PreStartContainer": (PreStartContainerRequest, PreStartContainerResponse, False),
}
DEVICE_PLUGIN_SERVICE = f"{PACKAGE}.DevicePlugin"
REGISTRATION_SERVICE = f"{PACKAGE}.Registration"


def add_device_plugin_servicer(server, servicer):
    import grpc

    handlers = {}
    for name, (req, resp, stream) in DEVICE_PLUGIN_METHODS.items():
        fn = getattr(servicer, name)
        if stream:
            handlers[name] = grpc.unary_stream_rpc_method_handler(
                fn, request_deserializer=req.FromString, response_serializer=resp.SerializeToString)
        else:
            handlers[name] = grpc.unary_unary_rpc_method_handler(
                fn, request_deserializer=req.FromString, response_serializer=resp.SerializeToString)
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(DEVICE_PLUGIN_SERVICE, handlers),))


def add_registration_servicer(server, servicer):
    import grpc

    h = grpc.unary_unary_rpc_method_handler(servicer.Register, request_deserializer=RegisterRequest.FromString,
                                            response_serializer=Empty.SerializeToString)
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(REGISTRATION_SERVICE, {"Register": h}),))


class DevicePluginStub:
    def __init__(self, channel):
        for name, (req, resp, stream) in DEVICE_PLUGIN_METHODS.items():
            path = f"/{DEVICE_PLUGIN_SERVICE}/{name}"
            if stream:
                setattr(self, name, channel.unary_stream(path, request_serializer=req.SerializeToString,
                                                         response_deserializer=resp.FromString))
            else:
                setattr(self, name, channel.unary_unary(path, request_serializer=req.SerializeToString,
                                                        response_deserializer=resp.FromString))


class RegistrationStub:
    def __init__(self, channel):
        self.Register = channel.unary_unary(f"/{REGISTRATION_SERVICE}/Register",
                                            request_serializer=RegisterRequest.SerializeToString,
                                            response_deserializer=Empty.FromString)
