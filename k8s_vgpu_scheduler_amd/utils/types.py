"""Annotation keys, labels, env names and policy names (pkg/util/types.go:19-99).

Keys are kept byte-identical to HAMi so existing tooling, dashboards and
pods written for HAMi keep working; AMD-specific additions are marked.
"""

ASSIGNED_TIME_ANNOTATION = "hami.io/vgpu-time"
ASSIGNED_NODE_ANNOTATION = "hami.io/vgpu-node"
BIND_TIME_ANNOTATION = "hami.io/bind-time"
DEVICE_BIND_PHASE = "hami.io/bind-phase"

DEVICE_BIND_ALLOCATING = "allocating"
DEVICE_BIND_FAILED = "failed"
DEVICE_BIND_SUCCESS = "success"

DEVICE_LIMIT = 100

NODE_NAME_ENV = "NODE_NAME"
# AMD analogues of CUDA_TASK_PRIORITY / GPU_CORE_UTILIZATION_POLICY (types.go:39-40)
TASK_PRIORITY_ENV = "HIP_TASK_PRIORITY"
CORE_LIMIT_SWITCH_ENV = "GPU_CORE_UTILIZATION_POLICY"

ROLE_LABEL = "hami.io/scheduler-role"
ROLE_LEADER = "leader"
ROLE_FOLLOWER = "follower"
COMPONENT_LABEL = "app.kubernetes.io/component"
COMPONENT_SCHEDULER = "hami-scheduler"
POD_GROUP_LABEL = "scheduling.x-k8s.io/pod-group"

NODE_POLICY_BINPACK = "binpack"
NODE_POLICY_SPREAD = "spread"
GPU_POLICY_BINPACK = "binpack"
GPU_POLICY_SPREAD = "spread"
GPU_POLICY_TOPOLOGY = "topology-aware"
GPU_POLICY_MUTEX = "mutex"
GPU_POLICY_NUMA = "numa"

NODE_POLICY_ANNOTATION = "hami.io/node-scheduler-policy"
GPU_POLICY_ANNOTATION = "hami.io/gpu-scheduler-policy"
SCORING_WEIGHTS_ANNOTATION = "hami.io/device-scoring-weights"

WEIGHT = 10

NODE_LOCK_KEY = "hami.io/mutex.lock"
NODE_LOCK_SEP = ","

DEVICE_CORDON_ANNOTATION = "hami.io/device-cordon"
