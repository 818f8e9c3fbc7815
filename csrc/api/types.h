// Typed, read-mostly views of the Kubernetes objects the scheduler consumes.
//
// Parsed once from the store's JSON documents (store/store.h). Field coverage
// follows what the reference's plugins read from core/v1 Pod/Node
// (vendor/k8s.io/api/core/v1/types.go), scheduling.sigs.k8s.io/v1alpha1
// PodGroup/ElasticQuota (apis/scheduling/v1alpha1/types.go:30-193),
// topology.node.k8s.io/v1alpha1 NodeResourceTopology, policy/v1 PDB and
// scheduling/v1 PriorityClass.
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <optional>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "api/resource.h"
#include "common/json.h"

namespace xsched {

// ---- well-known keys (Appendix A of SURVEY.md) ----
inline constexpr const char* kPodGroupLabel = "pod-group.scheduling.sigs.k8s.io";
inline constexpr const char* kDefaultSchedulerName = "default-scheduler";

// Timestamps are microseconds since the Unix epoch; 0 = unset.
using MicroTime = int64_t;
MicroTime parse_rfc3339(const std::string& s);
std::string format_rfc3339(MicroTime t);
MicroTime wall_now_us();

using StrMap = std::vector<std::pair<std::string, std::string>>;  // small, ordered
const std::string* strmap_get(const StrMap& m, std::string_view k);
StrMap strmap_from_json(const Json& j);

// An object's labels or annotations, shared between copies of the object
// until one of them changes (copy on write): the scheduler copies a Pod per
// assume and per bind confirmation, and the maps are rarely touched then.
class SharedStrMap {
 public:
  SharedStrMap() = default;
  SharedStrMap(StrMap m) { *this = std::move(m); }  // NOLINT(google-explicit-constructor)
  SharedStrMap(std::initializer_list<std::pair<std::string, std::string>> l) : SharedStrMap(StrMap(l)) {}
  SharedStrMap& operator=(StrMap m) {
    p_ = m.empty() ? nullptr : std::make_shared<StrMap>(std::move(m));
    return *this;
  }
  const StrMap& get() const { return p_ ? *p_ : none(); }
  operator const StrMap&() const { return get(); }  // NOLINT(google-explicit-constructor)
  StrMap::const_iterator begin() const { return get().begin(); }
  StrMap::const_iterator end() const { return get().end(); }
  size_t size() const { return p_ ? p_->size() : 0; }
  bool empty() const { return size() == 0; }
  // The map for writing: copied first when another object shares it. The
  // map is a non-const object (readers only ever see it through get()), so
  // writing through the sole owner is well-defined.
  StrMap& mut() {
    if (!p_) p_ = std::make_shared<StrMap>();
    else if (p_.use_count() > 1) p_ = std::make_shared<StrMap>(*p_);
    return *p_;
  }
  bool operator==(const SharedStrMap& o) const { return p_ == o.p_ || get() == o.get(); }
  bool operator!=(const SharedStrMap& o) const { return !(*this == o); }

 private:
  static const StrMap& none() {
    static const StrMap e;
    return e;
  }
  std::shared_ptr<StrMap> p_;
};

inline constexpr const char* kHostnameLabel = "kubernetes.io/hostname";

struct ObjectMeta {
  std::string ns, name, uid;
  int64_t resource_version = 0;
  SharedStrMap labels, annotations;
  MicroTime creation = 0;
  MicroTime deletion = 0;  // deletionTimestamp
  std::string key() const { return ns.empty() ? name : ns + "/" + name; }
  static ObjectMeta from_json(const Json& obj);
  const std::string* label(std::string_view k) const { return strmap_get(labels, k); }
  const std::string* annotation(std::string_view k) const { return strmap_get(annotations, k); }
};

// ---- selectors ----
enum class SelOp : uint8_t { In, NotIn, Exists, DoesNotExist, Gt, Lt };
struct SelectorRequirement {
  std::string key;
  SelOp op = SelOp::In;
  std::vector<std::string> values;
};
bool match_requirement(const SelectorRequirement& r, const StrMap& labels);

struct LabelSelector {  // metav1.LabelSelector
  bool present = false;  // nil selector matches nothing (PDB), empty matches all
  StrMap match_labels;
  std::vector<SelectorRequirement> exprs;
  bool matches(const StrMap& labels) const;
  static LabelSelector from_json(const Json* j);
};

struct NodeSelectorTerm {
  std::vector<SelectorRequirement> match_expressions;  // against node labels
  std::vector<SelectorRequirement> match_fields;       // metadata.name only
};
struct PreferredSchedulingTerm {
  int32_t weight = 0;
  NodeSelectorTerm pref;
};

struct Toleration {
  std::string key, op = "Equal", value, effect;
  int64_t toleration_seconds = -1;
  bool tolerates(const struct Taint& t) const;
};
struct Taint {
  std::string key, value, effect;  // NoSchedule, PreferNoSchedule, NoExecute
};

struct ContainerPort {
  int32_t host_port = 0;
  std::string protocol = "TCP", host_ip = "0.0.0.0";
};

struct Container {
  std::string name, image;
  Res requests, limits;
  std::vector<ContainerPort> ports;
};

// In-tree volume sources that count against per-node attach limits or can
// conflict between pods (VolumeRestrictions, the non-CSI limits plugins).
enum class InTree : uint8_t { None, AWSEBS, GCEPD, AzureDisk, Cinder, ISCSI, RBD };
const char* intree_plugin_name(InTree k);  // "kubernetes.io/aws-ebs", ... (api/storage.cc)

struct PodVolume {
  enum class Kind : uint8_t { Other, PVC, Ephemeral, InTree };
  std::string name;
  Kind kind = Kind::Other;
  std::string claim;  // PVC name (Ephemeral: "<pod>-<volume>")
  InTree intree = InTree::None;
  std::string id;     // EBS volumeID, GCE pdName, Azure diskName, Cinder volumeID, iSCSI IQN, RBD image
  bool read_only = false;
  std::vector<std::string> rbd_monitors;
  std::string rbd_pool;
};

// A vector fixed at parse time and shared by every copy of its object: the
// scheduler copies a Pod per scheduled pod (the assumed pod, the informer's
// bound object), and those copies then share the containers instead of
// duplicating their names, images and resource vectors.
template <typename T>
class SharedVec {
 public:
  SharedVec() = default;
  SharedVec(std::vector<T> v)  // NOLINT: implicit on purpose
      : p_(v.empty() ? nullptr : std::make_shared<const std::vector<T>>(std::move(v))) {}
  const std::vector<T>& get() const {
    static const std::vector<T> kEmpty;
    return p_ ? *p_ : kEmpty;
  }
  typename std::vector<T>::const_iterator begin() const { return get().begin(); }
  typename std::vector<T>::const_iterator end() const { return get().end(); }
  size_t size() const { return p_ ? p_->size() : 0; }
  bool empty() const { return !p_; }
  const T& operator[](size_t i) const { return (*p_)[i]; }

 private:
  std::shared_ptr<const std::vector<T>> p_;
};

enum class QoS : uint8_t { BestEffort = 0, Burstable = 1, Guaranteed = 2 };

struct PodAffinityTerm {
  LabelSelector selector;
  std::vector<std::string> namespaces;
  LabelSelector namespace_selector;  // present => also match namespaces by labels
  std::string topology_key;
};

// v1.TopologySpreadConstraint (k8s 1.23 fields).
struct TopologySpreadConstraint {
  int32_t max_skew = 1;
  std::string topology_key;
  bool hard = true;  // whenUnsatisfiable: DoNotSchedule (true) / ScheduleAnyway
  LabelSelector selector;
};

struct ContainerImage {
  std::vector<std::string> names;
  int64_t size_bytes = 0;
};
struct WeightedPodAffinityTerm {
  int32_t weight = 0;
  PodAffinityTerm term;
};

// GPU placement of a pod on an MI355X node, decoded from the FlexGPU
// annotations (plugins/flexgpu.cc documents the format).
struct GpuAssignment {
  enum class Kind : uint8_t { None, WholeGpu, Partition, Memory };
  Kind kind = Kind::None;
  std::vector<int> gpus;                           // physical GPU indexes
  std::vector<std::pair<int, int>> partitions;     // (gpu, partition) pairs
  int64_t memory = 0;                              // memory slice units
  bool valid() const { return kind != Kind::None; }
};

// What a pod asks of the FlexGPU plugin (decoded once at parse time).
struct GpuDemand {
  enum Kind : uint8_t { None, Gpu, Xcd, Memory, Conflict };
  Kind kind = None;
  int64_t amount = 0;
};

// An interned string: values from a small set (scheduler names, preemption
// policies) that every Pod copy would otherwise re-allocate (both exceed the
// 15-character small-string buffer). Copying is a pointer copy; the table
// lives for the process.
class IStr {
 public:
  IStr() : s_(&intern("")) {}
  IStr(std::string_view v) : s_(&intern(v)) {}  // NOLINT: implicit on purpose
  IStr(const char* v) : s_(&intern(v)) {}       // NOLINT
  IStr(const std::string& v) : s_(&intern(v)) {}  // NOLINT
  const std::string& str() const { return *s_; }
  operator const std::string&() const { return *s_; }  // NOLINT
  bool operator==(std::string_view v) const { return *s_ == v; }
  bool operator!=(std::string_view v) const { return *s_ != v; }
  bool empty() const { return s_->empty(); }
  static const std::string& intern(std::string_view v);

 private:
  const std::string* s_;
};

// An int64 field that one thread may update while others read it (relaxed:
// a timestamp, no ordering implied). Copyable, unlike std::atomic.
struct RelaxedI64 {
  std::atomic<int64_t> v{0};
  RelaxedI64() = default;
  RelaxedI64(int64_t x) : v(x) {}  // NOLINT: implicit on purpose
  RelaxedI64(const RelaxedI64& o) : v(o.v.load(std::memory_order_relaxed)) {}
  RelaxedI64& operator=(const RelaxedI64& o) {
    v.store(o.v.load(std::memory_order_relaxed), std::memory_order_relaxed);
    return *this;
  }
  RelaxedI64& operator=(int64_t x) {
    v.store(x, std::memory_order_relaxed);
    return *this;
  }
  operator int64_t() const { return v.load(std::memory_order_relaxed); }  // NOLINT
};

struct GpuNames;
const GpuNames& default_gpu_names();

// What a Pod asks for, derived once at parse time. Immutable and shared by
// the copies of a Pod (the scheduler copies a Pod per assume and per bind
// confirmation; four Res vectors are 1.5 KB of the object).
struct PodRes {
  Res request;          // computePodResourceRequest: max(sum(containers), each init) + overhead
  Res nonzero_request;  // cpu/memory with scheduler defaults for zero requests
  Res limit_sum;        // Σ container limits (FlexGPU accounting uses limits)
  Res overhead;         // spec.overhead
  static const std::shared_ptr<const PodRes>& empty() {
    static const std::shared_ptr<const PodRes> e = std::make_shared<const PodRes>();
    return e;
  }
};

struct Pod {
  ObjectMeta meta;
  IStr scheduler_name = kDefaultSchedulerName;
  std::string node_name, nominated_node_name, priority_class_name, phase = "Pending";
  IStr preemption_policy = "PreemptLowerPriority";
  int32_t priority = 0;
  SharedVec<Container> containers, init_containers;
  SharedVec<PodVolume> volumes;  // PVC / ephemeral / in-tree disk volumes (others are not parsed)
  StrMap node_selector;
  std::vector<NodeSelectorTerm> required_node_terms;  // OR of terms
  bool has_required_node_affinity = false;
  std::vector<PreferredSchedulingTerm> preferred_node_terms;
  std::vector<Toleration> tolerations;
  std::vector<PodAffinityTerm> pod_affinity_required, pod_anti_affinity_required;
  std::vector<WeightedPodAffinityTerm> pod_affinity_preferred, pod_anti_affinity_preferred;
  std::vector<TopologySpreadConstraint> spread_constraints;
  // status.startTime and the PodScheduled=True lastTransitionTime (0 = unset).
  // Relaxed atomics: a bind confirmation copies them into the assumed object
  // that NodeInfos (and Snapshot readers) already hold (cache.cc).
  RelaxedI64 start_time = 0;
  RelaxedI64 scheduled_at = 0;
  // The informer instance whose lister holds exactly this object (0: none
  // or superseded). Not copied: a copy is a different object.
  struct ListedMark {
    std::atomic<uint64_t> by{0};
    ListedMark() = default;
    ListedMark(const ListedMark&) {}
    ListedMark& operator=(const ListedMark&) { return *this; }
  };
  mutable ListedMark listed;
  // Which PodHeap holds exactly this object (PodHeap::tag; 0: none). Read and
  // written under the SchedulingQueue's lock only; not copied.
  struct HeapTag {
    uint8_t v = 0;
    HeapTag() = default;
    HeapTag(const HeapTag&) {}
    HeapTag& operator=(const HeapTag&) { return *this; }
  };
  mutable HeapTag heap_tag;

  // ---- derived at parse time ----
  // The resource vectors derived from the spec (PodRes), one immutable block
  // shared by every copy of the Pod.
  std::shared_ptr<const PodRes> res = PodRes::empty();
  const Res& request() const { return res->request; }
  const Res& nonzero_request() const { return res->nonzero_request; }
  const Res& limit_sum() const { return res->limit_sum; }
  const Res& overhead() const { return res->overhead; }
  QoS qos = QoS::BestEffort;
  std::string pod_group;  // value of kPodGroupLabel ("" if none)
  uint64_t pg_key = 0;    // pg_key_of("ns/pod_group"), 0 if no group
  std::vector<ContainerPort> host_ports;
  GpuAssignment gpu;      // decoded from annotations (mutable via cache only)
  GpuDemand gpu_demand;   // FlexGPU demand from container limits
  // Equivalence class: hash of namespace, annotations and spec (minus
  // nodeName). Pods with the same resource shape share it across PodGroups,
  // so Filter verdicts and Score values of node-local plugins can be reused.
  // Labels are left out on purpose: the only plugins that read a pod's labels
  // (InterPodAffinity, PodTopologySpread, XGMIGangAffinity via the PodGroup)
  // declare themselves non-local whenever those labels can matter.
  uint64_t template_hash = 0;
  // Hash of the spec minus nodeName: two objects of one pod with equal
  // spec_hash, labels and GPU assignment account identically on a node (the
  // cache keeps the assumed object when its bind is confirmed).
  uint64_t spec_hash = 0;

  const std::string& ns() const { return meta.ns; }
  const std::string& name() const { return meta.name; }
  const std::string& uid() const { return meta.uid; }
  std::string key() const { return meta.ns + "/" + meta.name; }
  bool terminating() const { return meta.deletion != 0; }
  std::string pg_full_name() const { return pod_group.empty() ? std::string() : meta.ns + "/" + pod_group; }

  static std::shared_ptr<Pod> from_json(const Json& obj, const GpuNames& gn = default_gpu_names());
  void recompute_gpu_assignment(const GpuNames& gn = default_gpu_names());
  // The assignment recompute_gpu_assignment derives from the index and
  // partition annotations, from already-parsed values (FlexGPU Reserve sets
  // the annotations and this together).
  void set_gpu_assignment(std::vector<int> gpus, std::vector<std::pair<int, int>> parts,
                          const GpuNames& gn = default_gpu_names());
};
using PodPtr = std::shared_ptr<Pod>;

// 64-bit key of a PodGroup full name "ns/name" (per-node gang counts).
uint64_t pg_key_of(std::string_view full_name);

struct Node {
  ObjectMeta meta;
  Res allocatable, capacity;
  bool unschedulable = false;
  std::vector<Taint> taints;
  std::vector<ContainerImage> images;  // status.images (ImageLocality)
  // Derived at parse time: every image name on the node -> size (first entry
  // wins, as upstream NodeInfo.ImageStates), and whether any taint is
  // PreferNoSchedule. The cache keeps cluster-wide counts of both.
  std::unordered_map<std::string, int64_t> image_sizes;
  bool has_prefer_no_schedule = false;
  // kubernetes.io/hostname label present and different from the node name:
  // then hostname topology domains may span nodes (see Snapshot).
  bool foreign_hostname = false;
  // MI355X GPU topology as published by the node agent (see flexgpu.cc).
  int gpu_count = 0;
  std::vector<int> gpu_partitions;  // partitions per physical GPU (1 = SPX .. 8 = CPX)
  std::vector<int> gpu_numa;        // NUMA node per GPU (-1 unknown)
  int64_t gpu_memory_per_gpu = 0;   // memory slice units per physical GPU
  const std::string& name() const { return meta.name; }
  static std::shared_ptr<Node> from_json(const Json& obj, const GpuNames& gn = default_gpu_names());
};
using NodePtr = std::shared_ptr<Node>;

// nodeSelector + required node affinity (nodeaffinity.GetRequiredNodeAffinity
// (pod).Match(node)); used by NodeAffinity and PodTopologySpread.
bool node_selector_term_matches(const NodeSelectorTerm& t, const Node& n);
bool pod_matches_node_selector_and_affinity(const Pod& p, const Node& n);

struct PodGroup {
  ObjectMeta meta;
  int32_t min_member = 0;
  bool has_min_resources = false;
  Res min_resources;
  int32_t schedule_timeout_seconds = -1;  // -1 = unset
  std::string phase, occupied_by;
  int32_t scheduled = 0, running = 0, succeeded = 0, failed = 0;
  MicroTime schedule_start_time = 0;
  // Set by the informer when a newer version replaces this object (or the
  // PodGroup is deleted): per-thread lookup caches drop it then.
  mutable RelaxedI64 superseded = 0;
  static std::shared_ptr<PodGroup> from_json(const Json& obj);
};
using PodGroupPtr = std::shared_ptr<PodGroup>;

struct ElasticQuota {
  ObjectMeta meta;
  Res min, max, used;
  bool has_min = false, has_max = false;
  static std::shared_ptr<ElasticQuota> from_json(const Json& obj);
};
using ElasticQuotaPtr = std::shared_ptr<ElasticQuota>;

struct NRTResourceInfo {
  std::string name;
  int64_t capacity = 0, allocatable = 0, available = 0;  // in scheduler units
  int res = -1;
};
struct NRTZone {
  std::string name, type;
  int numa_id = -1;  // parsed from "node-<id>"
  std::vector<NRTResourceInfo> resources;
  std::vector<std::pair<std::string, int64_t>> costs;
};
struct NumaZone {  // zone of type "Node" named node-<0..63>, available per resource
  int id = 0;
  std::vector<std::pair<int, int64_t>> res;  // (resource id, available)
  int64_t* find(int rid) {
    for (auto& kv : res)
      if (kv.first == rid) return &kv.second;
    return nullptr;
  }
  const int64_t* find(int rid) const { return const_cast<NumaZone*>(this)->find(rid); }
};
struct NodeResourceTopology {
  ObjectMeta meta;
  std::vector<std::string> topology_policies;
  std::vector<NRTZone> zones;
  std::vector<NumaZone> numa;  // precomputed createNUMANodeList, sorted by id
  static std::shared_ptr<NodeResourceTopology> from_json(const Json& obj);
};
using NRTPtr = std::shared_ptr<NodeResourceTopology>;

struct PodDisruptionBudget {
  ObjectMeta meta;
  LabelSelector selector;
  int32_t disruptions_allowed = 0;
  StrMap disrupted_pods;  // status.disruptedPods: pod name -> time
  static std::shared_ptr<PodDisruptionBudget> from_json(const Json& obj);
};
using PDBPtr = std::shared_ptr<PodDisruptionBudget>;

struct PriorityClass {
  ObjectMeta meta;
  int32_t value = 0;
  bool global_default = false;
  std::string preemption_policy;
  static std::shared_ptr<PriorityClass> from_json(const Json& obj);
};
using PriorityClassPtr = std::shared_ptr<PriorityClass>;

// GPU resource and annotation names used by pod/node parsing and the GPU
// plugins. Immutable once built; each Scheduler owns one, built from its
// profiles' FlexGPU args (the reference's package constants,
// pkg/flexgpu/flex_gpu.go:18-19, made configurable), and hands it to its
// informers, cache and plugins through the Handle. Two schedulers in one
// process may use different names; profiles of one scheduler share a cache
// (one GPU ledger per node), so they must agree.
struct GpuNames {
  std::string gpu = "amd.com/gpu";
  std::string memory = "amd.com/gpu-memory";
  std::string xcd = "amd.com/gpu-xcd";
  std::string index_annotation = "amd.com/gpu-index";
  std::string partition_annotation = "amd.com/gpu-partitions";
  std::string partition_label = "amd.com/gpu.compute-partition";     // spx|dpx|qpx|cpx
  std::string topology_annotation = "amd.com/gpu-topology";          // JSON, per-GPU detail

  GpuNames() { intern(); }
  // FlexGPU args (gpuResourceName, memoryResourceName, xcdResourceName,
  // indexAnnotationKey, partitionAnnotationKey) over the defaults.
  static std::shared_ptr<const GpuNames> from_args(const Json& args);
  bool operator==(const GpuNames& o) const {
    return gpu == o.gpu && memory == o.memory && xcd == o.xcd && index_annotation == o.index_annotation &&
           partition_annotation == o.partition_annotation;
  }
  std::string describe() const;
  // Interned resource ids (hot paths use these per node per pod).
  int gpu_id() const { return gpu_rid_; }
  int memory_id() const { return mem_rid_; }
  int xcd_id() const { return xcd_rid_; }

 private:
  void intern();
  int gpu_rid_ = -1, mem_rid_ = -1, xcd_rid_ = -1;
};
const GpuNames& default_gpu_names();
GpuDemand compute_gpu_demand(const Pod& p, const GpuNames& gn = default_gpu_names());
int partitions_for_mode(const std::string& mode);  // spx=1 dpx=2 qpx=4 cpx=8 (0 unknown)

}  // namespace xsched
