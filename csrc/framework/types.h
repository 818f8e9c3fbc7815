// Core framework value types: Status, CycleState, NodeInfo (+ the MI355X GPU
// ledger), Snapshot, QueuedPodInfo, ClusterEvent.
//
// Behavioural reference: vendor/k8s.io/kubernetes/pkg/scheduler/framework/
// {interface.go (Status codes), cycle_state.go, types.go (NodeInfo,
// QueuedPodInfo, ClusterEvent)} as used by the reference's plugins.
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <string>
#include <string_view>
#include <unordered_map>
#include <utility>
#include <vector>

#include "api/types.h"

namespace xsched {

// ------------------------------------------------------------- Status ----
enum class Code : uint8_t { Success = 0, Error, Unschedulable, UnschedulableAndUnresolvable, Wait, Skip };
const char* code_name(Code c);

// Copies are cheap (two refcounts): Filter returns a Status per node per
// plugin and the diagnosis keeps one per node, so failure reasons are shared,
// not re-allocated. Plugins keep their fixed failure statuses prebuilt.
class Status {
 public:
  Status() = default;
  // Copies only: a moved-from Status would keep a raw view of reasons its
  // owner took along, so moves copy (one reference count).
  Status(const Status&) = default;
  Status& operator=(const Status&) = default;
  explicit Status(Code c) : code_(c) {}
  Status(Code c, std::string reason)
      : code_(c), owner_(std::make_shared<const std::vector<std::string>>(1, std::move(reason))), reasons_(owner_.get()) {}
  Status(Code c, std::vector<std::string> reasons)
      : code_(c), owner_(std::make_shared<const std::vector<std::string>>(std::move(reasons))), reasons_(owner_.get()) {}
  static Status ok() { return Status(); }
  static Status error(std::string r) { return Status(Code::Error, std::move(r)); }
  static Status unschedulable(std::string r) { return Status(Code::Unschedulable, std::move(r)); }
  static Status unresolvable(std::string r) { return Status(Code::UnschedulableAndUnresolvable, std::move(r)); }
  // A failure built once for the life of the process (a plugin's fixed
  // Filter verdicts): copies share its reasons without a reference count, so
  // 16 Filter workers returning it for thousands of nodes never contend on
  // one atomic counter.
  static Status immortal(Code c, std::string reason) {
    Status s(c);
    s.reasons_ = new std::vector<std::string>(1, std::move(reason));  // never freed
    return s;
  }
  // An immortal failure shared process-wide per distinct (code, reasons):
  // plugins whose verdicts come from a small set (NodeResourcesFit's
  // "Insufficient <resource>" combinations, FlexGPU's per-resource failures)
  // memoize these, so the thousands of copies a failed cycle makes (one per
  // node into the diagnosis) never touch a reference count.
  static Status interned(Code c, std::vector<std::string> reasons);

  Code code() const { return code_; }
  bool is_success() const { return code_ == Code::Success; }
  bool is_wait() const { return code_ == Code::Wait; }
  bool is_skip() const { return code_ == Code::Skip; }
  bool is_unschedulable() const {
    return code_ == Code::Unschedulable || code_ == Code::UnschedulableAndUnresolvable;
  }
  const std::vector<std::string>& reasons() const;
  // Identity of the shared reasons list: statuses copied from one another
  // (e.g. a plugin's per-thread memo of a failure) compare equal here.
  const void* reasons_id() const { return reasons_; }
  const void* plugin_id() const { return plugin_; }
  std::string message() const;
  const std::string& failed_plugin() const;
  // Plugin names are interned (immortal), so a Status carries a plain pointer.
  Status& with_plugin(std::string_view p) {
    plugin_ = &intern_plugin(p);
    return *this;
  }
  Status& with_plugin(const std::string* interned) {
    plugin_ = interned;
    return *this;
  }
  static const std::string& intern_plugin(std::string_view p);

 private:
  Code code_ = Code::Success;
  std::shared_ptr<const std::vector<std::string>> owner_;  // empty for immortal statuses
  const std::vector<std::string>* reasons_ = nullptr;
  const std::string* plugin_ = nullptr;
};

// --------------------------------------------------------- CycleState ----
class StateData {
 public:
  virtual ~StateData() = default;
  virtual std::shared_ptr<StateData> clone() const = 0;
};

// Pods the current cycle wants moved to activeQ (framework.PodsToActivate).
struct PodsToActivate : StateData {
  std::mutex mu;
  // Duplicates are harmless: activating a pod already in activeQ is a no-op.
  std::vector<PodPtr> pods;
  std::shared_ptr<StateData> clone() const override { return nullptr; }  // shared, never cloned
};
inline constexpr const char* kPodsToActivateKey = "kubernetes.io/pods-to-activate";

// A PreFilter plugin's node set for this cycle (upstream's PreFilterResult,
// k8s 1.24+, by snapshot position instead of node name): the scheduler runs
// Filter only on these nodes and gives every other node `excluded`. When none
// of them passes Filter and `fallback` is set, every node is evaluated as if
// there were no restriction. Written under kNodeRestrictionKey.
struct NodeRestriction : StateData {
  size_t nodes = 0;        // snapshot size it was computed for (stale otherwise)
  std::vector<int> list;   // the allowed positions, when `mask` is empty
  std::vector<char> mask;  // per snapshot position (larger sets)
  bool fallback = true;
  Status excluded;         // verdict of the nodes outside the set
  bool allows(int pos) const {
    if (!mask.empty()) return mask[static_cast<size_t>(pos)] != 0;
    for (int q : list)
      if (q == pos) return true;
    return false;
  }
  std::shared_ptr<StateData> clone() const override { return std::make_shared<NodeRestriction>(*this); }
};
inline constexpr const char* kNodeRestrictionKey = "xsched/node-restriction";

// Node name -> pods nominated to it (Nominator::view()).
using NominatedMap = std::unordered_map<std::string, std::vector<PodPtr>>;

class CycleState {
 public:
  CycleState() : version_(next_version()) { kv_.reserve(8); }  // a cycle writes ~7 entries
  std::shared_ptr<StateData> read(std::string_view key) const;
  StateData* read_raw(std::string_view key) const;
  // Filter/Score run a plugin once per node on up to 16 threads against the
  // same CycleState; a per-thread memo (invalidated by any write, since every
  // write takes a fresh global version) turns the repeated lookup into two
  // loads instead of a mutex + refcount round-trip per node.
  template <typename T>
  T* read_as(std::string_view key) const {
    thread_local uint64_t memo_version = 0;
    thread_local std::string memo_key;
    thread_local T* memo = nullptr;
    uint64_t v = version_.load(std::memory_order_acquire);
    if (memo_version == v && memo_key == key) return memo;
    T* r = dynamic_cast<T*>(read_raw(key));
    memo_version = v;
    memo_key.assign(key.data(), key.size());
    memo = r;
    return r;
  }
  void write(std::string_view key, std::shared_ptr<StateData> v);
  void erase(std::string_view key);
  std::shared_ptr<CycleState> clone() const;
  bool record_metrics = false;
  bool skip_filter_plugins_mark = false;
  // Filter plugins (by position in the profile's Filter chain) that pass
  // every node for this cycle's pod (Plugin::skip_filter, evaluated once in
  // PreFilter): run_filter does not call them.
  uint64_t filter_skip = 0;
  // Nominated pods as of the cycle's start, shared read-only by the Filter
  // workers (null: ask the Nominator). Saves a lock and a vector copy per
  // node while preemptions keep nominations outstanding.
  std::shared_ptr<const NominatedMap> nominated;

 private:
  static uint64_t next_version();
  // Readers (Filter workers, preemption dry runs cloning the state per
  // candidate node on every worker) share the lock; only writes are exclusive.
  mutable std::shared_mutex mu_;
  std::atomic<uint64_t> version_;
  // Keys are interned (IStr): a clone copies pointers, not strings.
  std::vector<std::pair<const std::string*, std::shared_ptr<StateData>>> kv_;
};
using CycleStatePtr = std::shared_ptr<CycleState>;

// ----------------------------------------------------------- GpuLedger ----
// Per-node accounting of MI355X GPUs. A node has `gpu_count` physical GPUs;
// GPU g is split into parts[g] compute partitions (SPX=1, DPX=2, QPX=4,
// CPX=8; each partition owns 8/parts XCDs and mem_per_gpu/parts memory
// units). The ledger is updated incrementally as pods enter/leave the node,
// replacing the reference's per-call O(pods) rebuild (gpu_node.go:30-120).
struct GpuLedgerState {
  struct Slot {
    int exclusive = 0;     // whole-GPU or partition owners (expected 0/1)
    int64_t used_mem = 0;  // Σ memory-slice pods on this partition
    int mem_pods = 0;
  };
  int gpu_count = 0;
  int64_t mem_per_gpu = 0;
  std::vector<int> parts, offset;  // offset[g] = first slot of GPU g
  std::vector<int> monopoly;       // whole-GPU owners per GPU
  std::vector<int> numa;
  std::vector<Slot> slots;

  // Derived per-GPU availability, kept current by init()/apply() so Filter
  // and Score read O(#GPUs) or O(1) aggregates instead of walking slots.
  struct GpuFree {
    int whole = 0;         // 1 if an untouched SPX GPU
    int free_slots = 0;    // partitions with no owner and no memory use
    int xcds = 0;          // XCDs in those partitions
    int64_t mem = 0;       // free memory over non-exclusive partitions
    int64_t max_slot_mem = -1;  // largest free memory of one non-exclusive partition (-1: none)
  };
  static constexpr int kMaxZones = 64;
  std::vector<GpuFree> free;
  int tot_whole = 0, tot_xcds = 0;
  int64_t tot_mem = 0;
};

// Per-zone totals live in fixed arrays sized for the largest NUMA id; only
// the first zone_n entries (1 + the largest NUMA id of a GPU) are ever
// non-zero, so copies (every NodeInfo clone and preemption dry run) move
// those and not the 1.3 KB of the full arrays.
struct GpuLedger : GpuLedgerState {
  int zone_n = 0;
  int zone_gpus[kMaxZones] = {}, zone_whole[kMaxZones] = {}, zone_xcds[kMaxZones] = {};
  int64_t zone_mem[kMaxZones] = {};

  GpuLedger() = default;
  GpuLedger(const GpuLedger& o) : GpuLedgerState(o) { copy_zones(o); }
  GpuLedger& operator=(const GpuLedger& o) {
    if (this != &o) {
      GpuLedgerState::operator=(o);
      copy_zones(o);
    }
    return *this;
  }

  void init(const Node& n);
  void apply(const GpuAssignment& a, int sign);
  // Fields (by name) where this ledger's usage and derived availability
  // differ from `o` (cache debugger: incremental vs re-derived).
  std::vector<std::string> diff(const GpuLedger& o) const;
  int64_t part_mem(int g) const { return parts[g] > 0 ? mem_per_gpu / parts[g] : 0; }
  int xcds_per_part(int g) const { return parts[g] > 0 ? 8 / parts[g] : 0; }
  bool gpu_untouched(int g) const;      // no owner and no memory use on any partition
  // A whole-GPU claim needs an untouched GPU in SPX mode: on a partitioned
  // GPU the container would see 2/4/8 separate devices, not one MI355X.
  bool whole_gpu_free(int g) const { return free[g].whole != 0; }
  bool slot_free(int g, int p) const;   // exclusive-free and no memory use
  void copy_zones(const GpuLedger& o) {
    const int n = std::max(zone_n, o.zone_n);
    std::copy_n(o.zone_gpus, n, zone_gpus);
    std::copy_n(o.zone_whole, n, zone_whole);
    std::copy_n(o.zone_xcds, n, zone_xcds);
    std::copy_n(o.zone_mem, n, zone_mem);
    zone_n = o.zone_n;
  }
  int free_gpus() const { return tot_whole; }  // GPUScore (gpu_node.go:179-187): free whole (SPX) GPUs
  int64_t free_memory() const { return tot_mem; }  // MemScore (gpu_node.go:189-199)
  int free_xcds() const { return tot_xcds; }
  // Bit b set: some GPU without a whole-GPU owner is partitioned into
  // (1 << b)-XCD partitions (b = 0..3: CPX .. SPX).
  uint8_t part_mask() const {
    uint8_t m = 0;
    for (int g = 0; g < gpu_count; ++g) {
      const int x = xcds_per_part(g);
      if (monopoly[g] > 0 || x <= 0) continue;
      m |= static_cast<uint8_t>(x >= 8 ? 8 : x >= 4 ? 4 : x >= 2 ? 2 : 1);
    }
    return m;
  }

 private:
  GpuFree compute(int g) const;
  void refresh(int g);
};

// ------------------------------------------------------------ NodeInfo ----
struct NodeInfo {
  NodePtr node;
  std::vector<PodPtr> pods;
  // std::hash of each pod's uid, parallel to `pods`: remove_pod/find_pod scan
  // this contiguous array instead of dereferencing every pod (and its uid's
  // heap buffer) on the node.
  std::vector<uint64_t> pod_uid_hashes;
  std::vector<PodPtr> pods_with_affinity;
  std::vector<PodPtr> pods_with_required_anti_affinity;
  std::set<std::tuple<std::string, std::string, int32_t>> used_ports;  // (ip, proto, port)
  Res requested, nonzero_requested, allocatable;
  GpuLedger gpu;
  NRTPtr nrt;  // this node's NodeResourceTopology (set by the cache from the informer)
  int64_t generation = 0;
  // PodGroup key (Pod::pg_key) -> pods of that group on this node. A flat
  // vector: a node hosts few groups and NodeInfo versions are copied on write.
  std::vector<std::pair<uint64_t, int>> pg_count;
  int pg_pods(uint64_t key) const {
    for (const auto& [k, c] : pg_count)
      if (k == key) return c;
    return 0;
  }

  const std::string& name() const;
  void set_node(const NodePtr& n);
  void add_pod(const PodPtr& p);
  bool remove_pod(const std::string& uid);
  int num_pods() const { return static_cast<int>(pods.size()); }
  std::shared_ptr<NodeInfo> clone() const { return std::make_shared<NodeInfo>(*this); }
  const PodPtr* find_pod(const std::string& uid) const;
  // Fields where this NodeInfo's incremental accounting differs from one
  // rebuilt from scratch out of its Node and pods (cache debugger).
  std::vector<std::string> verify() const;
};
using NodeInfoPtr = std::shared_ptr<NodeInfo>;
// Nodes of one scheduling cycle (feasible set, score order). Borrowed from
// the Snapshot, which holds every version for the whole cycle, so the hot
// path passes raw pointers instead of bumping shared refcounts per node.
using NodeList = std::vector<const NodeInfo*>;

// One pod entering (+1) or leaving (-1) a node's NodeInfo, as the cache
// applied it, with the Node object of that moment. Plugins that count pods
// cluster-wide in PreFilter (PodTopologySpread, InterPodAffinity) replay the
// events since an earlier cycle to bring that cycle's state up to date
// instead of recounting every pod of every node.
struct PodDelta {
  PodPtr pod;
  NodePtr node;
  int d = 0;
};

// ------------------------------------------------------------ Snapshot ----
struct Snapshot {
  std::vector<NodeInfoPtr> nodes;  // in cache order
  // nodes[i]'s name, contiguous: the per-node loops of a failed cycle (the
  // FitError diagnosis over every node) read names without touching each
  // NodeInfo and Node.
  std::vector<std::string> names;
  std::unordered_map<std::string, NodeInfoPtr> by_name;
  std::unordered_map<std::string, size_t> index;  // name -> position in `nodes`
  // nodes[i]->generation, contiguous: equivalence-cache checks on the Filter
  // and Score paths compare generations without touching each NodeInfo.
  std::vector<int64_t> gen;
  // nodes[i]->gpu.free_gpus() (whole SPX GPUs free), contiguous likewise.
  std::vector<int32_t> free_whole;
  // nodes[i]->gpu.free_xcds() and .part_mask(), contiguous likewise (XCD gangs).
  std::vector<int32_t> free_xcd;
  std::vector<uint8_t> part_mask;
  // Cluster totals of the two arrays above, kept in step by set_gpu_summary:
  // free whole GPUs, and free XCDs per partition-size mask (Coscheduling's
  // gang gate reads them per cycle without a pass over the nodes).
  int64_t sum_free_whole = 0;
  int64_t sum_free_xcd_by_mask[16] = {};
  // `fresh`: the arrays were just resized for a rebuilt node list, so slot i
  // holds nothing to subtract (reset_gpu_sums() ran first).
  void set_gpu_summary(size_t i, bool fresh = false) {
    const GpuLedger& L = nodes[i]->gpu;
    if (!fresh) {
      sum_free_whole -= free_whole[i];
      sum_free_xcd_by_mask[part_mask[i] & 15] -= free_xcd[i];
    }
    gen[i] = nodes[i]->generation;
    free_whole[i] = L.free_gpus();
    free_xcd[i] = L.free_xcds();
    part_mask[i] = L.part_mask();
    sum_free_whole += free_whole[i];
    sum_free_xcd_by_mask[part_mask[i] & 15] += free_xcd[i];
  }
  void reset_gpu_sums() {
    sum_free_whole = 0;
    std::fill(std::begin(sum_free_xcd_by_mask), std::end(sum_free_xcd_by_mask), int64_t{0});
  }
  // Nodes with affinity / required anti-affinity pods, in no particular
  // order. Kept incrementally by the cache: *_pos[i] is node i's slot in the
  // list (-1 if absent) and *_idx the reverse, so a refresh touches only the
  // nodes that changed instead of rescanning every node.
  std::vector<NodeInfoPtr> have_pods_with_affinity;
  std::vector<NodeInfoPtr> have_pods_with_required_anti_affinity;
  std::vector<int32_t> affinity_pos, anti_pos;
  std::vector<uint32_t> affinity_idx, anti_idx;
  int64_t generation = 0;
  uint64_t node_epoch = 0;  // bumped on any Node object / node-set change (not on pod changes)
  // Nodes carrying at least one PreferNoSchedule taint, kept by the cache as
  // Nodes change. Zero lets TaintToleration skip its Score pass.
  int64_t nodes_with_prefer_no_schedule = 0;
  // Lowest priority of any pod on a node (INT32_MAX when none): a preemptor
  // at or below it has no possible lower-priority victim anywhere.
  int32_t min_pod_priority = INT32_MAX;
  // No node carries a kubernetes.io/hostname label other than its own name,
  // so a hostname topology domain is exactly one node: InterPodAffinity then
  // evaluates hostname-keyed anti-affinity on the node's own pods instead of
  // counting them cluster-wide in PreFilter.
  bool hostname_domains_are_nodes = true;
  // Image name -> number of nodes listing it (upstream ImageStateSummary.
  // NumNodes), published with the same refresh as `nodes`, so ImageLocality's
  // score and its all-zero skip read one consistent view. Never null.
  std::shared_ptr<const std::unordered_map<std::string, int64_t>> image_spread =
      std::make_shared<const std::unordered_map<std::string, int64_t>>();
  // Bumped when a node joins or leaves or its labels change: pod counts per
  // topology domain stay comparable across cycles while it holds.
  uint64_t topology_epoch = 0;
  // The most recent pod events (oldest first); delta_end is the sequence
  // number one past deltas.back().
  static constexpr size_t kMaxDeltas = 16384;
  std::deque<PodDelta> deltas;
  uint64_t delta_end = 0;
  // Set by a plugin that memoizes a state against delta_end (scheduling
  // thread); the cache records pod events only from the next refresh on.
  mutable bool deltas_wanted = false;
  // Calls fn(delta) for each pod event after sequence `from` (a delta_end
  // seen in an earlier cycle) and returns true, or returns false without
  // calling fn when some of them have been trimmed.
  template <typename Fn>
  bool replay_since(uint64_t from, Fn&& fn) const {
    if (from > delta_end || delta_end - from > deltas.size()) return false;
    for (size_t i = deltas.size() - static_cast<size_t>(delta_end - from); i < deltas.size(); ++i) fn(deltas[i]);
    return true;
  }
  // Versions replaced by the last refreshes (and trimmed pod events). Dropping
  // one can free deleted pods, so the scheduler releases them off the
  // scheduling thread.
  std::vector<NodeInfoPtr> retired;
  std::vector<PodDelta> retired_deltas;
  NodeInfoPtr get(const std::string& name) const {
    auto it = by_name.find(name);
    return it == by_name.end() ? nullptr : it->second;
  }
  bool has(const std::string& name) const { return by_name.count(name) != 0; }
};

// -------------------------------------------------------- QueuedPodInfo ----
struct QueuedPodInfo {
  PodPtr pod;
  int64_t timestamp_us = 0;          // last time added to a queue (monotonic)
  int64_t initial_attempt_us = 0;    // first time added (monotonic)
  MicroTime initial_attempt_wall = 0;
  int attempts = 0;
  std::set<std::string> unschedulable_plugins;
  // "message|nominated node" of the last failure whose PodScheduled=False
  // status was written (Scheduler::handle_failure skips identical rewrites).
  std::string last_condition;
  int64_t enqueue_seq = 0;
  // QueueSort plugins may memoize an immutable sort key here (e.g.
  // Coscheduling's PodGroup creation time); INT64_MIN = not cached.
  mutable int64_t sort_key_cache = INT64_MIN;
  // pod->priority, memoized for heap comparisons (valid while prio_of == pod.get()).
  mutable const Pod* prio_of = nullptr;
  mutable int32_t prio_cache = 0;
  int32_t priority() const {
    if (prio_of != pod.get()) {
      prio_cache = pod->priority;
      prio_of = pod.get();
    }
    return prio_cache;
  }
  // Position in the PodHeap currently holding this entry (a QueuedPodInfo
  // sits in at most one heap at a time); lets sift-up/down skip uid hashing.
  size_t heap_index = 0;
};
using QueuedPodInfoPtr = std::shared_ptr<QueuedPodInfo>;

// -------------------------------------------------------- ClusterEvent ----
enum ActionType : uint32_t {
  kAdd = 1, kDelete = 2, kUpdateNodeAllocatable = 4, kUpdateNodeLabel = 8, kUpdateNodeTaint = 16,
  kUpdateNodeCondition = 32, kUpdate = 4 | 8 | 16 | 32, kAll = 63
};
struct ClusterEvent {
  std::string resource;  // "Pod", "Node", "PodGroup", "ElasticQuota", "*" ...
  uint32_t action = kAll;
  std::string label;
  bool is_wildcard() const { return resource == "*" && action == kAll; }
  bool matches(const ClusterEvent& other) const {
    return is_wildcard() || (resource == other.resource && (action & other.action) != 0);
  }
};

// One node's score in a plugin row or the total row. `name` points at the
// NodeInfo's node name (stable for the cycle) and is set only where a reader
// needs it (explain, normalizers that declare normalize_uses_names), so a
// row is 16 trivially-copyable bytes per node.
struct NodeScore {
  const std::string* name = nullptr;
  int64_t score = 0;
};
inline constexpr int64_t kMaxNodeScore = 100;
inline constexpr int64_t kMinNodeScore = 0;

// Node name -> Filter status of one failed cycle (framework.NodeToStatusMap).
// A cycle that finds no node fills it with every node of the cluster before
// PostFilter, so it is a flat map: entries in one vector (insertion order)
// and an open-addressing index of positions, i.e. no allocation per node.
// The subset of the std::unordered_map interface the scheduler and the
// plugins use: find / count / emplace / operator[] / iteration / reserve.
class NodeStatusMap {
 public:
  using value_type = std::pair<std::string, Status>;
  using const_iterator = std::vector<value_type>::const_iterator;
  using iterator = std::vector<value_type>::iterator;

  NodeStatusMap() = default;
  NodeStatusMap(const NodeStatusMap& o) { *this = o; }
  NodeStatusMap& operator=(const NodeStatusMap& o) {
    if (this != &o) {
      o.ensure_index();
      entries_ = o.entries_;
      hashes_ = o.hashes_;
      slots_ = o.slots_;
      indexed_.store(o.indexed_.load(std::memory_order_acquire), std::memory_order_relaxed);
      clear_deferred();
    }
    return *this;
  }

  size_t size() const { return deferred() ? deferred_.size() : entries_.size(); }
  bool empty() const { return size() == 0; }
  const_iterator begin() const {
    materialize();
    return entries_.begin();
  }
  const_iterator end() const {
    materialize();
    return entries_.end();
  }
  iterator begin() {
    materialize();
    return entries_.begin();
  }
  iterator end() {
    materialize();
    return entries_.end();
  }
  void clear() {
    entries_.clear();
    hashes_.clear();
    slots_.clear();
    indexed_.store(0, std::memory_order_relaxed);
    clear_deferred();
  }
  void reserve(size_t n) { entries_.reserve(n); }
  const_iterator find(std::string_view k) const {
    ensure_index();
    int32_t i = lookup(k, hash(k));
    return i < 0 ? entries_.end() : entries_.begin() + i;
  }
  iterator find(std::string_view k) {
    ensure_index();
    int32_t i = lookup(k, hash(k));
    return i < 0 ? entries_.end() : entries_.begin() + i;
  }
  size_t count(std::string_view k) const { return status_of(k) ? 1 : 0; }
  std::pair<iterator, bool> emplace(std::string_view k, const Status& v) {
    ensure_index();
    const size_t h = hash(k);
    if (int32_t i = lookup(k, h); i >= 0) return {entries_.begin() + i, false};
    entries_.emplace_back(std::string(k), v);
    index_tail();
    return {entries_.end() - 1, true};
  }
  // Appends a node the caller knows is not in the map yet. Nothing is
  // hashed: the index is built on the first lookup by key.
  void append_unique(std::string_view k, const Status& v) {
    materialize();
    entries_.emplace_back(std::string(k), v);
  }
  Status& operator[](std::string_view k) { return emplace(k, Status()).first->second; }

  // ---- deferred form: what a failed scheduling cycle builds ----
  // (snapshot position, status) pairs naming the snapshot's nodes, with no
  // string or Status copied. Valid for the cycle that built them: `names`
  // and `pos_index` are the Snapshot's, the statuses live in the cycle's
  // Filter buffers. The first iteration, key lookup by iterator or copy
  // materializes owned entries; status_of / count_code / for_each do not,
  // and a PostFilter that only asks those (DefaultPreemption over 5,000
  // nodes) never pays the copy.
  void defer(const std::vector<std::string>* names, const std::unordered_map<std::string, size_t>* pos_index) {
    clear();
    def_names_ = names;
    def_index_ = pos_index;
    pos_to_def_.assign(names->size(), -1);
  }
  void append_deferred(int32_t pos, const Status* st) {
    pos_to_def_[pos] = static_cast<int32_t>(deferred_.size());
    deferred_.emplace_back(pos, st);
  }
  // The status recorded for node `k`, nullptr if none.
  const Status* status_of(std::string_view k) const {
    if (deferred()) {
      auto it = def_index_->find(std::string(k));
      if (it == def_index_->end() || it->second >= pos_to_def_.size()) return nullptr;
      int32_t i = pos_to_def_[it->second];
      return i < 0 ? nullptr : deferred_[i].second;
    }
    auto it = find(k);
    return it == entries_.end() ? nullptr : &it->second;
  }
  size_t count_code(Code c) const {
    size_t n = 0;
    for_each([&](std::string_view, const Status& st) { n += st.code() == c; });
    return n;
  }
  template <class F>
  void for_each(F&& f) const {
    if (deferred()) {
      for (const auto& [pos, st] : deferred_) f(std::string_view((*def_names_)[pos]), *st);
      return;
    }
    for (const auto& [k, st] : entries_) f(std::string_view(k), st);
  }

 private:
  bool deferred() const { return def_names_ != nullptr && !materialized_.load(std::memory_order_acquire); }
  void clear_deferred() {
    def_names_ = nullptr;
    def_index_ = nullptr;
    deferred_.clear();
    pos_to_def_.clear();
    materialized_.store(false, std::memory_order_relaxed);
  }
  void materialize() const {
    if (!deferred()) return;
    std::lock_guard<std::mutex> g(index_mu());
    if (!deferred()) return;
    entries_.reserve(entries_.size() + deferred_.size());
    for (const auto& [pos, st] : deferred_) entries_.emplace_back((*def_names_)[pos], *st);
    materialized_.store(true, std::memory_order_release);
  }
  static size_t hash(std::string_view k) { return std::hash<std::string_view>{}(k); }
  // Indexes entries appended since the last lookup. Lookups on a shared map
  // from several threads are safe: the first one to arrive builds the index
  // under a lock, the others see it complete.
  void ensure_index() const {
    materialize();
    if (indexed_.load(std::memory_order_acquire) == entries_.size()) return;
    std::lock_guard<std::mutex> g(index_mu());
    if (indexed_.load(std::memory_order_relaxed) == entries_.size()) return;
    index_tail();
  }
  void index_tail() const {
    size_t from = indexed_.load(std::memory_order_relaxed);
    if (entries_.size() * 2 > slots_.size()) {
      size_t cap = 16;
      while (cap < entries_.size() * 2) cap <<= 1;
      hashes_.resize(from);
      for (size_t i = from; i < entries_.size(); ++i) hashes_.push_back(hash(entries_[i].first));
      slots_.assign(cap, -1);
      for (int32_t i = 0; i < static_cast<int32_t>(entries_.size()); ++i) place(i, hashes_[i]);
    } else {
      for (size_t i = from; i < entries_.size(); ++i) {
        hashes_.push_back(hash(entries_[i].first));
        place(static_cast<int32_t>(i), hashes_[i]);
      }
    }
    indexed_.store(entries_.size(), std::memory_order_release);
  }
  static std::mutex& index_mu() {
    static std::mutex m;
    return m;
  }
  int32_t lookup(std::string_view k, size_t h) const {
    if (slots_.empty()) return -1;
    size_t mask = slots_.size() - 1;
    for (size_t j = h & mask;; j = (j + 1) & mask) {
      int32_t i = slots_[j];
      if (i < 0) return -1;
      if (hashes_[i] == h && entries_[i].first == k) return i;
    }
  }
  void place(int32_t i, size_t h) const {
    size_t mask = slots_.size() - 1;
    size_t j = h & mask;
    while (slots_[j] >= 0) j = (j + 1) & mask;
    slots_[j] = i;
  }
  mutable std::vector<value_type> entries_;
  // Index over entries_[0, indexed_): each key hashed once, kept beside the
  // entry, so probing compares hashes before strings.
  mutable std::vector<size_t> hashes_;
  mutable std::vector<int32_t> slots_;  // power of two, at most half full; -1 = empty
  mutable std::atomic<size_t> indexed_{0};
  // deferred form
  const std::vector<std::string>* def_names_ = nullptr;
  const std::unordered_map<std::string, size_t>* def_index_ = nullptr;
  std::vector<std::pair<int32_t, const Status*>> deferred_;
  std::vector<int32_t> pos_to_def_;
  mutable std::atomic<bool> materialized_{false};
};

struct Victims {
  std::vector<PodPtr> pods;
  int64_t num_pdb_violations = 0;
};

struct PostFilterResult {
  std::string nominated_node_name;
};

}  // namespace xsched
