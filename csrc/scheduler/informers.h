// Typed informer caches (listers) fed from the store's watch stream.
//
// Replaces the reference's generated listers/informers (pkg/generated/
// listers/scheduling/v1alpha1/*.go, client-go core listers) with one typed,
// RW-locked cache per kind plus the secondary indexes the plugins query on
// their hot paths: pods by (namespace, PodGroup label) — Coscheduling's
// PreFilter/ActivateSiblings list (pkg/coscheduling/core/core.go:111-167) —
// and ElasticQuotas by namespace (pkg/capacityscheduling/capacity_scheduling.go:703-708).
#pragma once

#include <atomic>

#include <map>
#include <memory>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "api/storage.h"
#include "api/types.h"

namespace xsched {

class Informers {
 public:
  // ---- mutation (informer thread) ----
  void upsert_pod(const PodPtr& p);
  void delete_pod(const Pod& p);
  void delete_pods(const std::vector<PodPtr>& ps);  // one lock for a run of deletions
  // upsert_pod for the non-null ps[0..n), one lock; prev[i] receives the
  // object each replaced (nullptr if none).
  void upsert_pods(const PodPtr* ps, PodPtr* prev, size_t n);
  // A run of Deleted events, one lock: removes each "ns/name" key and returns
  // the lister's object where it is the same pod (uid) on the same node, else
  // nullptr (the caller parses the event's final state).
  std::vector<PodPtr> take_pods(const std::vector<std::string>& keys, const std::vector<std::string_view>& uids,
                                const std::vector<std::string_view>& nodes);
  void upsert_pod_group(const PodGroupPtr& pg);
  void delete_pod_group(const std::string& key);
  void upsert_elastic_quota(const ElasticQuotaPtr& eq);
  void delete_elastic_quota(const std::string& key);
  void upsert_nrt(const NRTPtr& n);
  void delete_nrt(const std::string& name);
  void upsert_pdb(const PDBPtr& p);
  void delete_pdb(const std::string& key);
  void upsert_priority_class(const PriorityClassPtr& pc);
  void delete_priority_class(const std::string& name);
  // storage (core/v1 PV/PVC, storage.k8s.io/v1 StorageClass/CSINode)
  void upsert_pv(const PVPtr& pv);
  void delete_pv(const std::string& name);
  void upsert_pvc(const PVCPtr& pvc);
  void delete_pvc(const std::string& key);
  void upsert_storage_class(const StorageClassPtr& sc);
  void delete_storage_class(const std::string& name);
  void upsert_csinode(const CSINodePtr& n);
  void delete_csinode(const std::string& name);

  // ---- listers ----
  PodPtr pod(const std::string& ns, const std::string& name) const;
  std::vector<PodPtr> pods_in_group(const std::string& ns, const std::string& pg) const;
  size_t count_pods_in_group(const std::string& ns, const std::string& pg) const;
  // Members of p's PodGroup, found by p.pg_key (no key string built).
  std::vector<PodPtr> pods_in_group_of(const Pod& p) const;
  size_t count_pods_in_group_of(const Pod& p) const;
  std::vector<PodPtr> all_pods() const;
  PodGroupPtr pod_group(const std::string& ns, const std::string& name) const;
  // The PodGroup named by p's group label, looked up by p.pg_key (no string
  // building on the scheduling path).
  PodGroupPtr pod_group_of(const Pod& p) const;
  std::vector<PodGroupPtr> pod_groups() const;
  ElasticQuotaPtr elastic_quota_for_namespace(const std::string& ns) const;
  std::vector<ElasticQuotaPtr> elastic_quotas() const;
  NRTPtr nrt(const std::string& node) const;
  std::vector<PDBPtr> pdbs() const;
  PriorityClassPtr priority_class(const std::string& name) const;
  size_t pod_count() const;
  // True while `p` is the object this lister holds for its key (no lookup).
  bool lists(const Pod& p) const { return p.listed.by.load(std::memory_order_relaxed) == instance_; }
  PVPtr pv(const std::string& name) const;
  PVCPtr pvc(const std::string& ns, const std::string& name) const;
  StorageClassPtr storage_class(const std::string& name) const;
  CSINodePtr csinode(const std::string& name) const;
  // PVs of one storage class ("" = no class), as pvCache.ListPVs(class).
  std::vector<PVPtr> pvs_of_class(const std::string& cls) const;

 private:
  mutable std::shared_mutex mu_;
  // Distinguishes instances for per-thread caches (an address can be reused).
  const uint64_t instance_ = next_instance();
  static uint64_t next_instance() {
    static std::atomic<uint64_t> n{0};
    return ++n;
  }
  std::unordered_map<std::string, PodPtr> pods_;  // ns/name
  // PodGroup members by Pod::pg_key (64-bit hash of "ns/pg"). Readers still
  // compare namespace and group name, so a hash collision cannot mix groups.
  std::unordered_map<uint64_t, std::vector<PodPtr>> pods_by_group_;
  std::unordered_map<std::string, PodGroupPtr> pgs_;
  std::unordered_map<uint64_t, PodGroupPtr> pgs_by_key_;  // same objects, keyed by pg_key_of("ns/name")
  void group_remove(const PodPtr& p);
  std::map<std::string, ElasticQuotaPtr> eqs_;  // ordered: "first listed wins"
  std::unordered_map<std::string, NRTPtr> nrts_;
  std::unordered_map<std::string, PDBPtr> pdbs_;
  std::unordered_map<std::string, PriorityClassPtr> pcs_;
  std::unordered_map<std::string, PVPtr> pvs_;
  std::unordered_map<std::string, std::vector<PVPtr>> pvs_by_class_;
  std::unordered_map<std::string, PVCPtr> pvcs_;  // ns/name
  std::unordered_map<std::string, StorageClassPtr> scs_;
  std::unordered_map<std::string, CSINodePtr> csinodes_;
};

}  // namespace xsched
