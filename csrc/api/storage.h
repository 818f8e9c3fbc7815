// Storage objects the volume plugins read: core/v1 PersistentVolume and
// PersistentVolumeClaim, storage.k8s.io/v1 StorageClass and CSINode, and the
// volumes of a Pod.
//
// Field coverage follows what the k8s 1.23 volume plugins the reference
// enables by default consult (vendor/k8s.io/kubernetes/pkg/scheduler/apis/
// config/v1beta2/default_plugins.go:41-62,94-103): VolumeBinding
// (volumebinding/binder.go, pkg/controller/volume/persistentvolume/util),
// VolumeZone, VolumeRestrictions and NodeVolumeLimits (CSI and in-tree).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "api/types.h"

namespace xsched {

// Annotations of the volume binding protocol (pkg/controller/volume/
// persistentvolume/util/util.go).
inline constexpr const char* kAnnSelectedNode = "volume.kubernetes.io/selected-node";
inline constexpr const char* kAnnBindCompleted = "pv.kubernetes.io/bind-completed";
inline constexpr const char* kAnnBoundByController = "pv.kubernetes.io/bound-by-controller";
inline constexpr const char* kAnnStorageClassBeta = "volume.beta.kubernetes.io/storage-class";
inline constexpr const char* kAnnMigratedPlugins = "storage.alpha.kubernetes.io/migrated-plugins";
inline constexpr const char* kNotSupportedProvisioner = "kubernetes.io/no-provisioner";

// Parsed from pod.spec.volumes (Pod::from_json).
std::vector<PodVolume> parse_pod_volumes(const Json& spec, const std::string& pod_name);

struct PersistentVolume {
  ObjectMeta meta;
  std::string storage_class;  // spec.storageClassName, else the beta annotation
  int64_t capacity = 0;       // spec.capacity.storage, bytes
  std::vector<std::string> access_modes;
  std::string volume_mode = "Filesystem";
  std::string phase;          // status.phase
  bool has_claim_ref = false;
  std::string claim_ns, claim_name, claim_uid;
  bool has_node_affinity = false;
  std::vector<NodeSelectorTerm> node_affinity;  // required terms (ORed)
  std::string csi_driver, csi_handle;
  InTree intree = InTree::None;
  std::string intree_id;
  bool matches_node(const Node& n) const;  // volumeutil.CheckNodeAffinity
  static std::shared_ptr<PersistentVolume> from_json(const Json& obj);
};
using PVPtr = std::shared_ptr<const PersistentVolume>;

struct PersistentVolumeClaim {
  ObjectMeta meta;
  bool has_class = false;     // storageClassName (or the beta annotation) set
  std::string storage_class;
  std::string volume_name;
  int64_t request = 0;        // spec.resources.requests.storage, bytes
  std::vector<std::string> access_modes;
  std::string volume_mode = "Filesystem";
  LabelSelector selector;     // spec.selector (nil = none)
  std::string phase;          // status.phase
  std::string controller_uid, controller_kind;  // controlling ownerReference
  bool fully_bound() const {  // isPVCFullyBound
    return !volume_name.empty() && meta.annotation(kAnnBindCompleted) != nullptr;
  }
  const std::string* selected_node() const { return meta.annotation(kAnnSelectedNode); }
  static std::shared_ptr<PersistentVolumeClaim> from_json(const Json& obj);
};
using PVCPtr = std::shared_ptr<const PersistentVolumeClaim>;

struct TopologySelectorTerm {
  std::vector<std::pair<std::string, std::vector<std::string>>> exprs;  // key In values
};

struct StorageClass {
  ObjectMeta meta;
  std::string provisioner;
  bool wait_for_first_consumer = false;  // volumeBindingMode (apiserver default Immediate)
  bool binding_mode_set = false;
  std::vector<TopologySelectorTerm> allowed_topologies;
  bool topology_matches(const Node& n) const;  // v1helper.MatchTopologySelectorTerms
  static std::shared_ptr<StorageClass> from_json(const Json& obj);
};
using StorageClassPtr = std::shared_ptr<const StorageClass>;

struct CSINode {
  ObjectMeta meta;
  struct Driver {
    std::string name;
    bool has_count = false;
    int64_t count = 0;
  };
  std::vector<Driver> drivers;
  bool migrated(InTree k) const;  // the migrated-plugins annotation lists k's plugin
  static std::shared_ptr<CSINode> from_json(const Json& obj);
};
using CSINodePtr = std::shared_ptr<const CSINode>;

// GetCSIAttachLimitKey: "attachable-volumes-csi-<driver>", shortened with a
// SHA-1 suffix when longer than a resource name may be.
std::string csi_attach_limit_key(const std::string& driver);

}  // namespace xsched
