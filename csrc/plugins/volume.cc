// The volume plugin family of kube-scheduler 1.23, enabled by default in
// every profile of the reference (vendor/k8s.io/kubernetes/pkg/scheduler/
// apis/config/v1beta2/default_plugins.go:41-62,94-103):
//
//   VolumeRestrictions  Filter: inline GCE PD / AWS EBS / RBD / iSCSI disks a
//                       pod on the node already uses (volumerestrictions/
//                       volume_restrictions.go:64-229)
//   VolumeZone          Filter: zone/region labels of bound PVs against the
//                       node's (volumezone/volume_zone.go:78-173)
//   NodeVolumeLimits    Filter: CSI attach limits per driver from CSINode /
//                       node allocatable (nodevolumelimits/csi.go:77-336)
//   EBSLimits, GCEPDLimits, AzureDiskLimits, CinderLimits
//                       Filter: in-tree attach limits (nodevolumelimits/
//                       non_csi.go:200-550)
//   VolumeBinding       PreFilter / Filter / Reserve / Unreserve / PreBind:
//                       bound PVs' node affinity, WaitForFirstConsumer
//                       claims matched to PVs (smallest fit) or dynamically
//                       provisioned on the chosen node, assumed in a cache at
//                       Reserve and bound through the API at PreBind, which
//                       then waits for the PV controller (volumebinding/
//                       volume_binding.go:170-380, binder.go:262-1000,
//                       pkg/controller/volume/persistentvolume/util/util.go).
//
// Pods without the relevant volumes skip each plugin's Filter for the whole
// cycle (Plugin::skip_filter), so the default profile costs GPU gangs nothing.
// Not modelled (documented in docs/MIGRATION.md): in-tree to CSI migration
// translation (a PV of an in-tree type counts for the in-tree limit plugins,
// not NodeVolumeLimits, unless the node's CSINode lists its plugin as
// migrated), CSIStorageCapacity and the alpha ReadWriteOncePod and
// VolumeCapacityPriority gates (off in 1.23).
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <mutex>
#include <random>
#include <regex>
#include <set>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "api/storage.h"
#include "framework/plugin.h"
#include "scheduler/informers.h"

namespace xsched {

namespace {

constexpr const char* kErrDiskConflict = "node(s) had no available disk";
constexpr const char* kErrZoneConflict = "node(s) had no available volume zone";
constexpr const char* kErrMaxVolumeCount = "node(s) exceed max volume count";
constexpr const char* kErrBindConflict = "node(s) didn't find available persistent volumes to bind";
constexpr const char* kErrNodeConflict = "node(s) had volume node affinity conflict";
constexpr const char* kErrPVNotExist = "node(s) unavailable due to one or more pvc(s) bound to non-existent pv(s)";

bool has_claims(const Pod& p) {
  for (const auto& v : p.volumes)
    if (v.kind == PodVolume::Kind::PVC || v.kind == PodVolume::Kind::Ephemeral) return true;
  return false;
}

std::string quoted(const std::string& s) { return "\"" + s + "\""; }

// A per-process random prefix for volumes not provisioned yet (the
// reference's randomVolumeIDPrefix): unique per (namespace, claim).
const std::string& random_volume_prefix() {
  static const std::string p = [] {
    std::mt19937_64 rng(std::random_device{}());
    static const char* a = "abcdefghijklmnopqrstuvwxyz0123456789";
    std::string s;
    for (int i = 0; i < 32; ++i) s.push_back(a[rng() % 36]);
    return s;
  }();
  return p;
}

// All limits the node advertises through allocatable "attachable-volumes-*".
std::unordered_map<std::string, int64_t> allocatable_volume_limits(const Node& n) {
  std::unordered_map<std::string, int64_t> out;
  auto& reg = ResourceRegistry::get();
  for (uint64_t m = n.allocatable.mask; m; m &= m - 1) {
    int i = __builtin_ctzll(m);
    std::string name = reg.name(i);
    if (name.rfind("attachable-volumes-", 0) == 0) out[name] = n.allocatable.get(i);
  }
  return out;
}

// ephemeral.VolumeIsForPod
Status ephemeral_owned(const Pod& p, const PersistentVolumeClaim& c) {
  if (c.controller_uid != p.uid())
    return Status::unresolvable("PVC " + c.meta.ns + "/" + c.meta.name + " was not created for pod " + p.ns() + "/" +
                                p.name() + " (pod is not owner)");
  return {};
}

// ====================================================== VolumeRestrictions ===
bool conflicts(const PodVolume& v, const PodVolume& e) {
  if (v.intree != e.intree || v.intree == InTree::None) return false;
  switch (v.intree) {
    case InTree::GCEPD:
    case InTree::ISCSI:
      return v.id == e.id && !(v.read_only && e.read_only);
    case InTree::AWSEBS:
      return v.id == e.id;
    case InTree::RBD: {
      bool overlap = false;
      for (const auto& m : v.rbd_monitors)
        if (std::find(e.rbd_monitors.begin(), e.rbd_monitors.end(), m) != e.rbd_monitors.end()) overlap = true;
      return overlap && v.rbd_pool == e.rbd_pool && v.id == e.id && !(v.read_only && e.read_only);
    }
    default:
      return false;
  }
}

bool restricted(const PodVolume& v) {
  return v.intree == InTree::GCEPD || v.intree == InTree::AWSEBS || v.intree == InTree::RBD ||
         v.intree == InTree::ISCSI;
}

class VolumeRestrictions : public Plugin {
 public:
  VolumeRestrictions() : Plugin("VolumeRestrictions", kPreFilter | kFilter) {}
  bool skip_filter(const Pod& p) const override {
    for (const auto& v : p.volumes)
      if (restricted(v)) return false;
    return true;
  }
  // Depends only on the node's pods.
  bool filter_node_local(const Pod&, const Snapshot&) const override { return true; }
  Status filter(CycleState&, const Pod& p, const NodeInfo& ni) override {
    for (const auto& v : p.volumes) {
      if (!restricted(v)) continue;
      for (const auto& q : ni.pods)
        for (const auto& e : q->volumes)
          if (conflicts(v, e)) return XS_FIXED_STATUS(Code::Unschedulable, kErrDiskConflict);
    }
    return {};
  }
  std::vector<ClusterEvent> events_to_register() const override {
    return {{"Pod", kDelete, ""}, {"Node", kAdd, ""}, {"PersistentVolumeClaim", kAdd | kUpdate, ""}};
  }
  std::vector<std::string> watched_kinds() const override { return {"persistentvolumeclaims"}; }
};

// ============================================================== VolumeZone ===
bool zone_label(std::string_view k) {
  return k == "failure-domain.beta.kubernetes.io/zone" || k == "failure-domain.beta.kubernetes.io/region" ||
         k == "topology.kubernetes.io/zone" || k == "topology.kubernetes.io/region";
}

// volumehelpers.LabelZonesToSet: "a__b__c".
bool zone_set_has(const std::string& v, const std::string& want) {
  size_t start = 0;
  while (start <= v.size()) {
    size_t end = v.find("__", start);
    if (end == std::string::npos) end = v.size();
    if (v.compare(start, end - start, want) == 0) return true;
    if (end == v.size()) break;
    start = end + 2;
  }
  return false;
}

class VolumeZone : public Plugin {
 public:
  explicit VolumeZone(Handle& h) : Plugin("VolumeZone", kFilter), h_(h) {}
  bool skip_filter(const Pod& p) const override {
    for (const auto& v : p.volumes)
      if (v.kind == PodVolume::Kind::PVC) return false;
    return true;
  }
  Status filter(CycleState&, const Pod& p, const NodeInfo& ni) override {
    const Node& node = *ni.node;
    StrMap constraints;
    for (const auto& [k, v] : node.meta.labels)
      if (zone_label(k)) constraints.emplace_back(k, v);
    if (constraints.empty()) return {};
    for (const auto& v : p.volumes) {
      if (v.kind != PodVolume::Kind::PVC) continue;
      if (v.claim.empty()) return Status::unresolvable("PersistentVolumeClaim had no name");
      PVCPtr pvc = h_.informers->pvc(p.ns(), v.claim);
      if (!pvc) return Status::unresolvable("persistentvolumeclaim " + quoted(v.claim) + " not found");
      if (pvc->volume_name.empty()) {
        if (!pvc->has_class || pvc->storage_class.empty())
          return Status::unresolvable("PersistentVolumeClaim had no pv name and storageClass name");
        StorageClassPtr sc = h_.informers->storage_class(pvc->storage_class);
        if (!sc) return Status::unresolvable("storageclass.storage.k8s.io " + quoted(pvc->storage_class) + " not found");
        if (!sc->binding_mode_set)
          return Status::unresolvable("VolumeBindingMode not set for StorageClass " + quoted(pvc->storage_class));
        if (sc->wait_for_first_consumer) continue;
        return Status::unresolvable("PersistentVolume had no name");
      }
      PVPtr pv = h_.informers->pv(pvc->volume_name);
      if (!pv) return Status::unresolvable("persistentvolume " + quoted(pvc->volume_name) + " not found");
      for (const auto& [k, val] : pv->meta.labels) {
        if (!zone_label(k)) continue;
        const std::string* nv = strmap_get(constraints, k);
        if (!zone_set_has(val, nv ? *nv : std::string()))
          return XS_FIXED_STATUS(Code::UnschedulableAndUnresolvable, kErrZoneConflict);
      }
    }
    return {};
  }
  std::vector<ClusterEvent> events_to_register() const override {
    return {{"StorageClass", kAdd, ""},
            {"Node", kAdd | kUpdateNodeLabel, ""},
            {"PersistentVolumeClaim", kAdd, ""},
            {"PersistentVolume", kAdd | kUpdate, ""}};
  }
  std::vector<std::string> watched_kinds() const override {
    return {"persistentvolumes", "persistentvolumeclaims", "storageclasses"};
  }

 private:
  Handle& h_;
};

// ======================================================== NodeVolumeLimits ===
bool migratable_provisioner(const std::string& p) {
  return p == "kubernetes.io/aws-ebs" || p == "kubernetes.io/gce-pd" || p == "kubernetes.io/azure-disk" ||
         p == "kubernetes.io/cinder" || p == "kubernetes.io/azure-file" || p == "kubernetes.io/vsphere-volume" ||
         p == "kubernetes.io/portworx-volume" || p == "kubernetes.io/rbd";
}

class CSILimits : public Plugin {
 public:
  explicit CSILimits(Handle& h) : Plugin("NodeVolumeLimits", kFilter), h_(h) {}
  bool skip_filter(const Pod& p) const override { return !has_claims(p); }
  Status filter(CycleState&, const Pod& p, const NodeInfo& ni) override {
    const Node& node = *ni.node;
    CSINodePtr csi = h_.informers->csinode(node.name());
    std::unordered_map<std::string, std::string> fresh;  // unique volume -> limit key
    if (Status st = attachable(p, csi.get(), true, fresh); !st.is_success()) return st;
    if (fresh.empty()) return {};
    auto limits = allocatable_volume_limits(node);
    if (csi)
      for (const auto& d : csi->drivers)
        if (d.has_count) limits[csi_attach_limit_key(d.name)] = d.count;
    if (limits.empty()) return {};
    std::unordered_map<std::string, std::string> attached;
    for (const auto& q : ni.pods) (void)attachable(*q, csi.get(), false, attached);
    std::unordered_map<std::string, int> attached_count, new_count;
    for (const auto& [vol, key] : attached) {
      fresh.erase(vol);
      ++attached_count[key];
    }
    for (const auto& [vol, key] : fresh) ++new_count[key];
    for (const auto& [key, n] : new_count) {
      auto it = limits.find(key);
      if (it != limits.end() && attached_count[key] + n > it->second)
        return XS_FIXED_STATUS(Code::Unschedulable, kErrMaxVolumeCount);
    }
    return {};
  }
  std::vector<ClusterEvent> events_to_register() const override {
    return {{"CSINode", kAdd, ""}, {"Pod", kDelete, ""}};
  }
  std::vector<std::string> watched_kinds() const override {
    return {"persistentvolumes", "persistentvolumeclaims", "storageclasses", "csinodes"};
  }

 private:
  Status attachable(const Pod& p, const CSINode* csi, bool new_pod,
                    std::unordered_map<std::string, std::string>& out) const {
    for (const auto& v : p.volumes) {
      if (v.kind != PodVolume::Kind::PVC && v.kind != PodVolume::Kind::Ephemeral) continue;
      if (v.claim.empty()) return Status::error("PersistentVolumeClaim had no name");
      PVCPtr pvc = h_.informers->pvc(p.ns(), v.claim);
      if (!pvc) {
        if (new_pod)
          return Status::error("looking up PVC " + p.ns() + "/" + v.claim + ": persistentvolumeclaim " + quoted(v.claim) +
                               " not found");
        continue;
      }
      if (v.kind == PodVolume::Kind::Ephemeral)
        if (Status st = ephemeral_owned(p, *pvc); !st.is_success()) return Status::error(st.message());
      auto [driver, handle] = driver_info(csi, *pvc);
      if (driver.empty() || handle.empty()) continue;
      out[driver + "/" + handle] = csi_attach_limit_key(driver);
    }
    return {};
  }
  std::pair<std::string, std::string> driver_info(const CSINode* csi, const PersistentVolumeClaim& pvc) const {
    if (!pvc.volume_name.empty())
      if (PVPtr pv = h_.informers->pv(pvc.volume_name)) {
        if (!pv->csi_driver.empty()) return {pv->csi_driver, pv->csi_handle};
        return {};  // in-tree source: no CSI translation here
      }
    if (!pvc.has_class || pvc.storage_class.empty()) return {};
    StorageClassPtr sc = h_.informers->storage_class(pvc.storage_class);
    if (!sc) return {};
    if (migratable_provisioner(sc->provisioner)) return {};  // migration not modelled
    return {sc->provisioner, random_volume_prefix() + "-" + pvc.meta.ns + "/" + pvc.meta.name};
  }
  Handle& h_;
};

class NonCSILimits : public Plugin {
 public:
  NonCSILimits(const char* name, InTree kind, std::string limit_key, Handle& h)
      : Plugin(name, kFilter), kind_(kind), limit_key_(std::move(limit_key)), h_(h) {}
  bool skip_filter(const Pod& p) const override { return p.volumes.empty(); }
  Status filter(CycleState&, const Pod& p, const NodeInfo& ni) override {
    std::unordered_set<std::string> fresh;
    if (Status st = volumes_of(p, true, fresh); !st.is_success()) return st;
    if (fresh.empty()) return {};
    const Node& node = *ni.node;
    if (CSINodePtr csi = h_.informers->csinode(node.name()); csi && csi->migrated(kind_)) return {};
    std::unordered_set<std::string> existing;
    for (const auto& q : ni.pods) (void)volumes_of(*q, false, existing);
    for (const auto& e : existing) fresh.erase(e);
    int64_t max = max_volumes(node);
    if (auto lim = allocatable_volume_limits(node); lim.count(limit_key_)) max = lim[limit_key_];
    if (static_cast<int64_t>(existing.size() + fresh.size()) > max)
      return XS_FIXED_STATUS(Code::Unschedulable, kErrMaxVolumeCount);
    return {};
  }
  std::vector<ClusterEvent> events_to_register() const override { return {{"Node", kAdd, ""}, {"Pod", kDelete, ""}}; }
  std::vector<std::string> watched_kinds() const override {
    return {"persistentvolumes", "persistentvolumeclaims", "storageclasses", "csinodes"};
  }

 private:
  Status volumes_of(const Pod& p, bool new_pod, std::unordered_set<std::string>& out) const {
    for (const auto& v : p.volumes) {
      if (v.kind == PodVolume::Kind::InTree) {
        if (v.intree == kind_) out.insert(v.id);
        continue;
      }
      if (v.kind != PodVolume::Kind::PVC && v.kind != PodVolume::Kind::Ephemeral) continue;
      if (v.claim.empty()) return Status::error("PersistentVolumeClaim had no name");
      std::string pv_id = random_volume_prefix() + "-" + p.ns() + "/" + v.claim;
      PVCPtr pvc = h_.informers->pvc(p.ns(), v.claim);
      if (!pvc) {
        if (new_pod)
          return Status::error("looking up PVC " + p.ns() + "/" + v.claim + ": persistentvolumeclaim " + quoted(v.claim) +
                               " not found");
        continue;
      }
      if (v.kind == PodVolume::Kind::Ephemeral)
        if (Status st = ephemeral_owned(p, *pvc); !st.is_success()) return Status::error(st.message());
      PVPtr pv = pvc->volume_name.empty() ? nullptr : h_.informers->pv(pvc->volume_name);
      if (!pv) {
        if (matches_provisioner(*pvc)) out.insert(pv_id);
        continue;
      }
      if (pv->intree == kind_) out.insert(pv->intree_id);
    }
    return {};
  }
  bool matches_provisioner(const PersistentVolumeClaim& pvc) const {
    if (!pvc.has_class) return false;
    StorageClassPtr sc = h_.informers->storage_class(pvc.storage_class);
    return sc && sc->provisioner == intree_plugin_name(kind_);
  }
  int64_t max_volumes(const Node& n) const {
    if (const char* env = std::getenv("KUBE_MAX_PD_VOLS")) {
      char* end = nullptr;
      long v = std::strtol(env, &end, 10);
      if (end && *end == '\0' && v > 0) return v;
    }
    switch (kind_) {
      case InTree::AWSEBS: {
        const std::string* t = n.meta.label("node.kubernetes.io/instance-type");
        if (!t) t = n.meta.label("beta.kubernetes.io/instance-type");
        static const std::regex nitro("^[cmr]5.*|t3|z1d");
        return t && std::regex_search(*t, nitro) ? 25 : 39;
      }
      case InTree::GCEPD: return 16;
      case InTree::AzureDisk: return 16;
      case InTree::Cinder: return 256;
      default: return INT64_MAX;
    }
  }
  InTree kind_;
  std::string limit_key_;
  Handle& h_;
};

// =========================================================== VolumeBinding ===
struct PodVolumes {
  std::vector<std::pair<PVCPtr, PVPtr>> bindings;  // static: claim -> matched (then assumed) PV
  std::vector<PVCPtr> provisions;                  // dynamic: claims (then assumed with selected-node)
};

struct VolumeBindingState : StateData {
  std::vector<PVCPtr> bound;    // fully bound claims
  std::vector<PVCPtr> to_bind;  // unbound WaitForFirstConsumer claims, smallest request first
  std::unordered_map<std::string, std::vector<PVPtr>> pvs;  // candidate PVs per class, with assumed ones
  std::mutex mu;
  std::unordered_map<std::string, std::shared_ptr<PodVolumes>> by_node;
  bool all_bound = true;
  std::shared_ptr<PodVolumes> reserved;
  // Shared across clones, as upstream's stateData.Clone returns itself.
  std::shared_ptr<StateData> clone() const override { return nullptr; }
};
constexpr const char* kVolumeBindingKey = "VolumeBinding";

bool bound_to_claim(const PersistentVolume& pv, const PersistentVolumeClaim& c) {
  if (!pv.has_claim_ref) return false;
  if (pv.claim_name != c.meta.name || pv.claim_ns != c.meta.ns) return false;
  return pv.claim_uid.empty() || pv.claim_uid == c.meta.uid;
}

bool access_modes_ok(const PersistentVolumeClaim& c, const PersistentVolume& pv) {
  for (const auto& m : c.access_modes)
    if (std::find(pv.access_modes.begin(), pv.access_modes.end(), m) == pv.access_modes.end()) return false;
  return true;
}

// pvutil.FindMatchingVolume, scheduler path (node set, delayBinding).
PVPtr find_matching_volume(const PersistentVolumeClaim& c, const std::vector<PVPtr>& pvs, const Node& node,
                           const std::unordered_set<std::string>& excluded) {
  PVPtr smallest;
  const std::string cls = c.has_class ? c.storage_class : "";
  for (const auto& pv : pvs) {
    if (excluded.count(pv->meta.name)) continue;
    if (pv->has_claim_ref && !bound_to_claim(*pv, c)) continue;
    if (pv->capacity < c.request) continue;
    if (pv->volume_mode != c.volume_mode) continue;
    if (pv->meta.deletion != 0) continue;
    const bool affinity_ok = pv->matches_node(node);
    if (bound_to_claim(*pv, c)) return affinity_ok ? pv : nullptr;  // pre-bound to this claim
    if (pv->phase != "Available") continue;
    if (c.selector.present && !c.selector.matches(pv->meta.labels)) continue;
    if (pv->storage_class != cls) continue;
    if (!affinity_ok) continue;
    if (!access_modes_ok(c, *pv)) continue;
    if (!smallest || pv->capacity < smallest->capacity) smallest = pv;
  }
  return smallest;
}

class VolumeBinding : public Plugin {
 public:
  VolumeBinding(const Json& args, Handle& h)
      : Plugin("VolumeBinding", kPreFilter | kFilter | kScore | kReserve | kPreBind), h_(h) {
    bind_timeout_us_ = args["bindTimeoutSeconds"].as_int(600) * 1'000'000;
    poll_us_ = std::max<int64_t>(1000, args["pollIntervalMillis"].as_int(100) * 1000);
  }

  bool skip_filter(const Pod& p) const override { return !has_claims(p); }
  // Score is the alpha VolumeCapacityPriority's (off in 1.23): 0 on every node,
  // so the framework never runs it.
  bool score_all_zero(const Pod&, const Snapshot&) const override { return true; }
  bool score_node_local(const Pod&, const Snapshot&) const override { return true; }

  Status pre_filter(CycleState& s, const Pod& p) override {
    if (!has_claims(p)) return {};
    auto st = std::make_shared<VolumeBindingState>();
    std::vector<PVCPtr> immediate;
    for (const auto& v : p.volumes) {
      if (v.kind != PodVolume::Kind::PVC && v.kind != PodVolume::Kind::Ephemeral) continue;
      const bool eph = v.kind == PodVolume::Kind::Ephemeral;
      PVCPtr pvc = get_pvc(p.ns(), v.claim);
      if (!pvc) {
        if (eph)
          return Status::unresolvable("waiting for ephemeral volume controller to create the persistentvolumeclaim " +
                                      quoted(v.claim));
        return Status::unresolvable("persistentvolumeclaim " + quoted(v.claim) + " not found");
      }
      if (pvc->phase == "Lost")
        return Status::unresolvable("persistentvolumeclaim " + quoted(pvc->meta.name) +
                                    " bound to non-existent persistentvolume " + quoted(pvc->volume_name));
      if (pvc->meta.deletion != 0)
        return Status::unresolvable("persistentvolumeclaim " + quoted(pvc->meta.name) + " is being deleted");
      if (eph)
        if (Status o = ephemeral_owned(p, *pvc); !o.is_success()) return o;
      if (pvc->fully_bound()) {
        st->bound.push_back(pvc);
        continue;
      }
      bool delay = false;
      if (pvc->has_class && !pvc->storage_class.empty()) {
        if (StorageClassPtr sc = h_.informers->storage_class(pvc->storage_class)) {
          if (!sc->binding_mode_set)
            return Status::error("VolumeBindingMode not set for StorageClass " + quoted(pvc->storage_class));
          delay = sc->wait_for_first_consumer;
        }
      }
      if (delay && pvc->volume_name.empty())
        st->to_bind.push_back(pvc);
      else
        immediate.push_back(pvc);  // immediate binding (or pre-bound): the PV controller's job
    }
    if (!immediate.empty()) return Status::unresolvable("pod has unbound immediate PersistentVolumeClaims");
    std::stable_sort(st->to_bind.begin(), st->to_bind.end(),
                     [](const PVCPtr& a, const PVCPtr& b) { return a->request < b->request; });
    for (const auto& c : st->to_bind) {
      std::string cls = c->has_class ? c->storage_class : "";
      if (!st->pvs.count(cls)) st->pvs[cls] = list_pvs(cls);
    }
    st->all_bound = false;
    s.write(kVolumeBindingKey, st);
    return {};
  }

  Status filter(CycleState& s, const Pod& p, const NodeInfo& ni) override {
    auto* st = s.read_as<VolumeBindingState>(kVolumeBindingKey);
    if (!st) return {};
    const Node& node = *ni.node;
    bool bound_ok = true, unbound_ok = true, pvs_found = true;
    auto pv_out = std::make_shared<PodVolumes>();
    auto reasons = [&]() {
      std::vector<std::string> r;
      if (!bound_ok) r.push_back(kErrNodeConflict);
      if (!unbound_ok) r.push_back(kErrBindConflict);
      if (!pvs_found) r.push_back(kErrPVNotExist);
      return r;
    };
    for (const auto& c : st->bound) {
      PVPtr pv = get_pv(c->volume_name);
      if (!pv) {
        pvs_found = false;
        break;
      }
      if (!pv->matches_node(node)) {
        bound_ok = false;
        break;
      }
    }
    if (!st->to_bind.empty()) {
      std::vector<PVCPtr> matching, provision;
      for (const auto& c : st->to_bind) {
        const std::string* sel = c->selected_node();
        if (sel) {
          if (*sel != node.name()) {  // fast path: provisioning already started elsewhere
            unbound_ok = false;
            return Status(Code::UnschedulableAndUnresolvable, reasons());
          }
          provision.push_back(c);
        } else {
          matching.push_back(c);
        }
      }
      if (!matching.empty()) {
        std::unordered_set<std::string> chosen;
        for (const auto& c : matching) {
          const auto& cands = st->pvs[c->has_class ? c->storage_class : ""];
          PVPtr pv = find_matching_volume(*c, cands, node, chosen);
          if (!pv) {
            unbound_ok = false;
            provision.push_back(c);
            continue;
          }
          chosen.insert(pv->meta.name);
          pv_out->bindings.emplace_back(c, pv);
        }
      }
      if (!provision.empty()) {
        unbound_ok = true;
        for (const auto& c : provision) {
          if (!c->has_class || c->storage_class.empty())
            return Status::error("no class for claim " + quoted(c->meta.key()));
          StorageClassPtr sc = h_.informers->storage_class(c->storage_class);
          if (!sc) return Status::error("failed to find storage class " + quoted(c->storage_class));
          if (sc->provisioner.empty() || sc->provisioner == kNotSupportedProvisioner || !sc->topology_matches(node)) {
            unbound_ok = false;
            pv_out->provisions.clear();
            break;
          }
          pv_out->provisions.push_back(c);
        }
      }
    }
    std::vector<std::string> r = reasons();
    if (!r.empty()) return Status(Code::UnschedulableAndUnresolvable, std::move(r));
    std::lock_guard<std::mutex> g(st->mu);
    st->by_node[node.name()] = std::move(pv_out);
    return {};
  }

  Status reserve(CycleState& s, const PodPtr& p, const std::string& node) override {
    auto* st = s.read_as<VolumeBindingState>(kVolumeBindingKey);
    if (!st) return {};
    std::shared_ptr<PodVolumes> pv;
    {
      std::lock_guard<std::mutex> g(st->mu);
      auto it = st->by_node.find(node);
      if (it != st->by_node.end()) pv = it->second;
    }
    st->all_bound = true;
    if (!pv || pod_volumes_bound(*p)) return {};
    auto assumed = std::make_shared<PodVolumes>();
    for (const auto& [c, vol] : pv->bindings) {
      PVPtr nv = vol;
      if (!(vol->has_claim_ref && vol->claim_name == c->meta.name && vol->claim_ns == c->meta.ns &&
            vol->claim_uid == c->meta.uid)) {
        auto copy = std::make_shared<PersistentVolume>(*vol);
        const bool prebound = bound_to_claim(*vol, *c);
        copy->has_claim_ref = true;
        copy->claim_ns = c->meta.ns;
        copy->claim_name = c->meta.name;
        copy->claim_uid = c->meta.uid;
        if (!prebound && !copy->meta.annotation(kAnnBoundByController))
          copy->meta.annotations.mut().emplace_back(kAnnBoundByController, "yes");
        nv = copy;
        assume_pv(nv);
      }
      assumed->bindings.emplace_back(c, nv);
    }
    for (const auto& c : pv->provisions) {
      auto copy = std::make_shared<PersistentVolumeClaim>(*c);
      bool set = false;
      StrMap& am = copy->meta.annotations.mut();
      for (auto& [k, v] : am)
        if (k == kAnnSelectedNode) {
          v = node;
          set = true;
        }
      if (!set) am.emplace_back(kAnnSelectedNode, node);
      assume_pvc(copy);
      assumed->provisions.push_back(copy);
    }
    st->reserved = assumed;
    st->all_bound = false;
    return {};
  }

  void unreserve(CycleState& s, const PodPtr&, const std::string&) override {
    auto* st = s.read_as<VolumeBindingState>(kVolumeBindingKey);
    if (!st || !st->reserved) return;
    revert(*st->reserved);
  }

  Status pre_bind(CycleState& s, const PodPtr& p, const std::string& node) override {
    auto* st = s.read_as<VolumeBindingState>(kVolumeBindingKey);
    if (!st || st->all_bound) return {};
    if (!st->reserved) return Status::error("no pod volumes found for node " + quoted(node));
    const PodVolumes& pv = *st->reserved;
    // bindAPIUpdate: the claim reference on each matched PV, the selected
    // node on each claim to provision; the PV controller does the rest.
    size_t done_b = 0, done_p = 0;
    try {
      for (const auto& [c, vol] : pv.bindings) {
        Json ref = Json::object();
        ref.set("kind", Json("PersistentVolumeClaim"));
        ref.set("apiVersion", Json("v1"));
        ref.set("namespace", Json(c->meta.ns));
        ref.set("name", Json(c->meta.name));
        ref.set("uid", Json(c->meta.uid));
        Json spec = Json::object();
        spec.set("claimRef", std::move(ref));
        Json patch = Json::object();
        patch.set("spec", std::move(spec));
        if (const std::string* a = vol->meta.annotation(kAnnBoundByController)) {
          Json ann = Json::object();
          ann.set(kAnnBoundByController, Json(*a));
          Json md = Json::object();
          md.set("annotations", std::move(ann));
          patch.set("metadata", std::move(md));
        }
        h_.client->patch("persistentvolumes", "", vol->meta.name, patch);
        ++done_b;
      }
      for (const auto& c : pv.provisions) {
        Json ann = Json::object();
        ann.set(kAnnSelectedNode, Json(node));
        Json md = Json::object();
        md.set("annotations", std::move(ann));
        Json patch = Json::object();
        patch.set("metadata", std::move(md));
        h_.client->patch("persistentvolumeclaims", c->meta.ns, c->meta.name, patch);
        ++done_p;
      }
    } catch (const std::exception& e) {
      PodVolumes rest;
      rest.bindings.assign(pv.bindings.begin() + static_cast<long>(done_b), pv.bindings.end());
      rest.provisions.assign(pv.provisions.begin() + static_cast<long>(done_p), pv.provisions.end());
      revert(rest);
      return Status::error(e.what());
    }
    // checkBindings until the PV controller has finished (wait.Poll). The
    // wait can last bindTimeoutSeconds: it holds a binder thread, so the
    // pool is told (upstream blocks one goroutine per pod instead).
    std::string err0;
    if (check_bindings(*p, node, pv, &err0) && err0.empty()) return {};
    if (!err0.empty()) return Status::error("binding volumes: " + err0);
    struct Blocking {
      const Handle& h;
      explicit Blocking(const Handle& hh) : h(hh) {
        if (h.blocking_begin) h.blocking_begin();
      }
      ~Blocking() {
        if (h.blocking_end) h.blocking_end();
      }
    } blocking(h_);
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(bind_timeout_us_);
    for (;;) {
      std::string err;
      bool done = check_bindings(*p, node, pv, &err);
      if (!err.empty()) return Status::error("binding volumes: " + err);
      if (done) return {};
      if (std::chrono::steady_clock::now() >= deadline)
        return Status::error("binding volumes: timed out waiting for the condition");
      std::this_thread::sleep_for(std::chrono::microseconds(poll_us_));
    }
  }

  std::vector<ClusterEvent> events_to_register() const override {
    return {{"StorageClass", kAdd | kUpdate, ""},
            {"PersistentVolumeClaim", kAdd | kUpdate, ""},
            {"PersistentVolume", kAdd | kUpdate, ""},
            {"Node", kAdd | kUpdateNodeLabel, ""},
            {"CSINode", kAdd | kUpdate, ""}};
  }
  std::vector<std::string> watched_kinds() const override {
    return {"persistentvolumes", "persistentvolumeclaims", "storageclasses", "csinodes"};
  }

 private:
  // ---- assume cache (volumebinding/assume_cache.go): an assumed object
  // shadows the informer's until the informer has a newer version.
  struct Assumed {
    std::shared_ptr<const void> obj;
    int64_t base_rv = 0;
  };
  PVPtr get_pv(const std::string& name) {
    PVPtr inf = h_.informers->pv(name);
    std::lock_guard<std::mutex> g(mu_);
    auto it = assumed_pvs_.find(name);
    if (it == assumed_pvs_.end()) return inf;
    if (inf && inf->meta.resource_version > it->second.base_rv) {
      assumed_pvs_.erase(it);
      return inf;
    }
    return std::static_pointer_cast<const PersistentVolume>(it->second.obj);
  }
  PVCPtr get_pvc(const std::string& ns, const std::string& name) {
    PVCPtr inf = h_.informers->pvc(ns, name);
    std::lock_guard<std::mutex> g(mu_);
    auto it = assumed_pvcs_.find(ns + "/" + name);
    if (it == assumed_pvcs_.end()) return inf;
    if (inf && inf->meta.resource_version > it->second.base_rv) {
      assumed_pvcs_.erase(it);
      return inf;
    }
    return std::static_pointer_cast<const PersistentVolumeClaim>(it->second.obj);
  }
  std::vector<PVPtr> list_pvs(const std::string& cls) {
    std::vector<PVPtr> out = h_.informers->pvs_of_class(cls);
    std::lock_guard<std::mutex> g(mu_);
    if (assumed_pvs_.empty()) return out;
    for (auto& pv : out) {
      auto it = assumed_pvs_.find(pv->meta.name);
      if (it != assumed_pvs_.end() && pv->meta.resource_version <= it->second.base_rv)
        pv = std::static_pointer_cast<const PersistentVolume>(it->second.obj);
    }
    return out;
  }
  void assume_pv(const PVPtr& pv) {
    std::lock_guard<std::mutex> g(mu_);
    assumed_pvs_[pv->meta.name] = Assumed{pv, pv->meta.resource_version};
  }
  void assume_pvc(const PVCPtr& c) {
    std::lock_guard<std::mutex> g(mu_);
    assumed_pvcs_[c->meta.key()] = Assumed{c, c->meta.resource_version};
  }
  void revert(const PodVolumes& pv) {
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& b : pv.bindings) assumed_pvs_.erase(b.second->meta.name);
    for (const auto& c : pv.provisions) assumed_pvcs_.erase(c->meta.key());
  }

  bool pod_volumes_bound(const Pod& p) {
    for (const auto& v : p.volumes) {
      if (v.kind != PodVolume::Kind::PVC && v.kind != PodVolume::Kind::Ephemeral) continue;
      PVCPtr c = get_pvc(p.ns(), v.claim);
      if (!c || !c->fully_bound()) return false;
    }
    return true;
  }

  // checkBindings, on the API objects (the informer store), not the cache.
  bool check_bindings(const Pod& p, const std::string& node_name, const PodVolumes& pv, std::string* err) {
    if (!h_.lookup) {
      *err = "no object lookup";
      return false;
    }
    if (!h_.lookup("pods", p.ns(), p.name())) {
      *err = "pod does not exist any more";
      return false;
    }
    JsonPtr nj = h_.lookup("nodes", "", node_name);
    if (!nj) {
      *err = "failed to get node " + quoted(node_name);
      return false;
    }
    NodePtr node = Node::from_json(*nj);
    for (const auto& [c, vol] : pv.bindings) {
      JsonPtr vj = h_.lookup("persistentvolumes", "", vol->meta.name);
      JsonPtr cj = h_.lookup("persistentvolumeclaims", c->meta.ns, c->meta.name);
      if (!vj || !cj) {
        *err = "failed to check binding: " + std::string(!vj ? "pv " + vol->meta.name : "pvc " + c->meta.key()) +
               " not found";
        return false;
      }
      auto api_pv = PersistentVolume::from_json(*vj);
      if (!api_pv->matches_node(*node)) {
        *err = "pv " + quoted(api_pv->meta.name) + " node affinity doesn't match node " + quoted(node_name);
        return false;
      }
      if (!api_pv->has_claim_ref || api_pv->claim_uid.empty()) {
        // Our own claimRef patch may not have landed in the store yet.
        if (api_pv->meta.resource_version <= vol->meta.resource_version) return false;
        *err = "ClaimRef got reset for pv " + quoted(api_pv->meta.name);
        return false;
      }
      if (!PersistentVolumeClaim::from_json(*cj)->fully_bound()) return false;
    }
    for (const auto& c : pv.provisions) {
      JsonPtr cj = h_.lookup("persistentvolumeclaims", c->meta.ns, c->meta.name);
      if (!cj) {
        *err = "failed to check provisioning pvc: pvc " + c->meta.key() + " not found";
        return false;
      }
      auto api = PersistentVolumeClaim::from_json(*cj);
      const std::string* sel = api->selected_node();
      if ((!sel || *sel != node_name) && api->meta.resource_version <= c->meta.resource_version)
        return false;  // our selected-node patch has not reached the informer store yet
      if (!sel || *sel != node_name) {
        *err = "provisioning failed for PVC " + quoted(api->meta.name);
        return false;
      }
      if (!api->volume_name.empty()) {
        JsonPtr vj = h_.lookup("persistentvolumes", "", api->volume_name);
        if (!vj) return false;  // the PV may not have propagated yet
        auto api_pv = PersistentVolume::from_json(*vj);
        if (!api_pv->matches_node(*node)) {
          *err = "pv " + quoted(api_pv->meta.name) + " node affinity doesn't match node " + quoted(node_name);
          return false;
        }
      }
      if (!api->fully_bound()) return false;
    }
    return true;
  }

  Handle& h_;
  int64_t bind_timeout_us_ = 600'000'000;
  int64_t poll_us_ = 100'000;
  std::mutex mu_;
  std::unordered_map<std::string, Assumed> assumed_pvs_;   // name
  std::unordered_map<std::string, Assumed> assumed_pvcs_;  // ns/name
};

PluginRegistrar r1("VolumeRestrictions", [](const Json&, Handle&) { return std::make_shared<VolumeRestrictions>(); });
PluginRegistrar r2("VolumeZone", [](const Json&, Handle& h) { return std::make_shared<VolumeZone>(h); });
PluginRegistrar r3("NodeVolumeLimits", [](const Json&, Handle& h) { return std::make_shared<CSILimits>(h); });
PluginRegistrar r4("EBSLimits", [](const Json&, Handle& h) {
  return std::make_shared<NonCSILimits>("EBSLimits", InTree::AWSEBS, "attachable-volumes-aws-ebs", h);
});
PluginRegistrar r5("GCEPDLimits", [](const Json&, Handle& h) {
  return std::make_shared<NonCSILimits>("GCEPDLimits", InTree::GCEPD, "attachable-volumes-gce-pd", h);
});
PluginRegistrar r6("AzureDiskLimits", [](const Json&, Handle& h) {
  return std::make_shared<NonCSILimits>("AzureDiskLimits", InTree::AzureDisk, "attachable-volumes-azure-disk", h);
});
PluginRegistrar r7("CinderLimits", [](const Json&, Handle& h) {
  return std::make_shared<NonCSILimits>("CinderLimits", InTree::Cinder, "attachable-volumes-cinder", h);
});
PluginRegistrar r8("VolumeBinding", [](const Json& a, Handle& h) { return std::make_shared<VolumeBinding>(a, h); });

}  // namespace

void link_volume_plugins() {}

}  // namespace xsched
