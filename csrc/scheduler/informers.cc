#include "scheduler/informers.h"

#include <mutex>

namespace xsched {

void Informers::group_remove(const PodPtr& p) {
  auto git = pods_by_group_.find(p->pg_key);
  if (git == pods_by_group_.end()) return;
  auto& v = git->second;
  for (size_t i = 0; i < v.size(); ++i)
    if (v[i] == p) {
      v[i] = std::move(v.back());
      v.pop_back();
      break;
    }
  if (v.empty()) pods_by_group_.erase(git);
}

void Informers::upsert_pod(const PodPtr& p) {
  std::unique_lock<std::shared_mutex> g(mu_);
  auto [it, fresh] = pods_.try_emplace(p->key(), p);
  if (!fresh) {
    if (it->second->pg_key) group_remove(it->second);
    if (it->second != p) it->second->listed.by.store(0, std::memory_order_relaxed);
    it->second = p;
  }
  p->listed.by.store(instance_, std::memory_order_relaxed);
  if (p->pg_key) pods_by_group_[p->pg_key].push_back(p);
}

void Informers::upsert_pods(const PodPtr* ps, PodPtr* prev, size_t n) {
  std::unique_lock<std::shared_mutex> g(mu_);
  for (size_t i = 0; i < n; ++i) {
    const PodPtr& p = ps[i];
    if (!p) continue;
    auto [it, fresh] = pods_.try_emplace(p->key(), p);
    if (!fresh) {
      prev[i] = it->second;
      if (it->second->pg_key) group_remove(it->second);
      if (it->second != p) it->second->listed.by.store(0, std::memory_order_relaxed);
      it->second = p;
    }
    p->listed.by.store(instance_, std::memory_order_relaxed);
    if (p->pg_key) pods_by_group_[p->pg_key].push_back(p);
  }
}

void Informers::delete_pod(const Pod& p) {
  std::unique_lock<std::shared_mutex> g(mu_);
  auto it = pods_.find(p.key());
  if (it == pods_.end()) return;
  if (it->second->pg_key) group_remove(it->second);
  it->second->listed.by.store(0, std::memory_order_relaxed);
  pods_.erase(it);
}

void Informers::delete_pods(const std::vector<PodPtr>& ps) {
  std::unique_lock<std::shared_mutex> g(mu_);
  for (const auto& p : ps) {
    auto it = pods_.find(p->key());
    if (it == pods_.end()) continue;
    if (it->second->pg_key) group_remove(it->second);
    it->second->listed.by.store(0, std::memory_order_relaxed);
    pods_.erase(it);
  }
}

std::vector<PodPtr> Informers::take_pods(const std::vector<std::string>& keys, const std::vector<std::string_view>& uids,
                                         const std::vector<std::string_view>& nodes) {
  std::vector<PodPtr> out(keys.size());
  std::unique_lock<std::shared_mutex> g(mu_);
  for (size_t k = 0; k < keys.size(); ++k) {
    auto it = pods_.find(keys[k]);
    if (it == pods_.end()) continue;
    PodPtr p = std::move(it->second);
    if (p->pg_key) group_remove(p);
    p->listed.by.store(0, std::memory_order_relaxed);
    pods_.erase(it);
    if (p->uid() == uids[k] && p->node_name == nodes[k]) out[k] = std::move(p);
  }
  return out;
}

void Informers::upsert_pod_group(const PodGroupPtr& pg) {
  std::unique_lock<std::shared_mutex> g(mu_);
  std::string key = pg->meta.key();
  pgs_by_key_[pg_key_of(key)] = pg;
  auto& slot = pgs_[std::move(key)];
  if (slot && slot != pg) slot->superseded = 1;
  slot = pg;
}
void Informers::delete_pod_group(const std::string& key) {
  std::unique_lock<std::shared_mutex> g(mu_);
  auto it = pgs_by_key_.find(pg_key_of(key));
  if (it != pgs_by_key_.end() && it->second->meta.key() == key) pgs_by_key_.erase(it);
  auto pit = pgs_.find(key);
  if (pit != pgs_.end()) {
    pit->second->superseded = 1;
    pgs_.erase(pit);
  }
}
void Informers::upsert_elastic_quota(const ElasticQuotaPtr& eq) {
  std::unique_lock<std::shared_mutex> g(mu_);
  eqs_[eq->meta.key()] = eq;
}
void Informers::delete_elastic_quota(const std::string& key) {
  std::unique_lock<std::shared_mutex> g(mu_);
  eqs_.erase(key);
}
void Informers::upsert_nrt(const NRTPtr& n) {
  std::unique_lock<std::shared_mutex> g(mu_);
  nrts_[n->meta.name] = n;
}
void Informers::delete_nrt(const std::string& name) {
  std::unique_lock<std::shared_mutex> g(mu_);
  nrts_.erase(name);
}
void Informers::upsert_pdb(const PDBPtr& p) {
  std::unique_lock<std::shared_mutex> g(mu_);
  pdbs_[p->meta.key()] = p;
}
void Informers::delete_pdb(const std::string& key) {
  std::unique_lock<std::shared_mutex> g(mu_);
  pdbs_.erase(key);
}
void Informers::upsert_priority_class(const PriorityClassPtr& pc) {
  std::unique_lock<std::shared_mutex> g(mu_);
  pcs_[pc->meta.name] = pc;
}
void Informers::delete_priority_class(const std::string& name) {
  std::unique_lock<std::shared_mutex> g(mu_);
  pcs_.erase(name);
}

PodPtr Informers::pod(const std::string& ns, const std::string& name) const {
  thread_local std::string key;  // no key allocation per lookup
  key.assign(ns);
  key.push_back('/');
  key.append(name);
  std::shared_lock<std::shared_mutex> g(mu_);
  auto it = pods_.find(key);
  return it == pods_.end() ? nullptr : it->second;
}

namespace {
uint64_t group_hash(const std::string& ns, const std::string& pg) {
  std::string full;
  full.reserve(ns.size() + 1 + pg.size());
  full.append(ns).push_back('/');
  full.append(pg);
  return pg_key_of(full);
}
}  // namespace

std::vector<PodPtr> Informers::pods_in_group(const std::string& ns, const std::string& pg) const {
  std::vector<PodPtr> out;
  const uint64_t key = group_hash(ns, pg);
  std::shared_lock<std::shared_mutex> g(mu_);
  auto git = pods_by_group_.find(key);
  if (git == pods_by_group_.end()) return out;
  out.reserve(git->second.size());
  for (const auto& p : git->second)
    if (p->pod_group == pg && p->ns() == ns) out.push_back(p);
  return out;
}

size_t Informers::count_pods_in_group(const std::string& ns, const std::string& pg) const {
  const uint64_t key = group_hash(ns, pg);
  std::shared_lock<std::shared_mutex> g(mu_);
  auto git = pods_by_group_.find(key);
  if (git == pods_by_group_.end()) return 0;
  size_t n = 0;
  for (const auto& p : git->second) n += p->pod_group == pg && p->ns() == ns;
  return n;
}

std::vector<PodPtr> Informers::pods_in_group_of(const Pod& p) const {
  std::vector<PodPtr> out;
  if (!p.pg_key) return out;
  std::shared_lock<std::shared_mutex> g(mu_);
  auto git = pods_by_group_.find(p.pg_key);
  if (git == pods_by_group_.end()) return out;
  out.reserve(git->second.size());
  for (const auto& q : git->second)
    if (q->pod_group == p.pod_group && q->ns() == p.ns()) out.push_back(q);
  return out;
}

size_t Informers::count_pods_in_group_of(const Pod& p) const {
  if (!p.pg_key) return 0;
  std::shared_lock<std::shared_mutex> g(mu_);
  auto git = pods_by_group_.find(p.pg_key);
  if (git == pods_by_group_.end()) return 0;
  size_t n = 0;
  for (const auto& q : git->second) n += q->pod_group == p.pod_group && q->ns() == p.ns();
  return n;
}

std::vector<PodPtr> Informers::all_pods() const {
  std::shared_lock<std::shared_mutex> g(mu_);
  std::vector<PodPtr> out;
  out.reserve(pods_.size());
  for (const auto& kv : pods_) out.push_back(kv.second);
  return out;
}

size_t Informers::pod_count() const {
  std::shared_lock<std::shared_mutex> g(mu_);
  return pods_.size();
}

PodGroupPtr Informers::pod_group(const std::string& ns, const std::string& name) const {
  std::shared_lock<std::shared_mutex> g(mu_);
  auto it = pgs_.find(ns + "/" + name);
  return it == pgs_.end() ? nullptr : it->second;
}

PodGroupPtr Informers::pod_group_of(const Pod& p) const {
  if (!p.pg_key) return nullptr;
  // Consecutive cycles schedule the members of one gang, and every cycle
  // looks its PodGroup up several times (PreFilter, PreScore, Permit, gang
  // metrics): a per-thread last-hit entry, valid until the informer
  // supersedes the object, skips the shared lock and the map.
  struct Last {
    uint64_t owner = 0;
    uint64_t key = 0;
    PodGroupPtr pg;
  };
  thread_local Last last;
  if (last.owner == instance_ && last.key == p.pg_key && last.pg && last.pg->superseded.v.load(std::memory_order_relaxed) == 0 &&
      last.pg->meta.name == p.pod_group && last.pg->meta.ns == p.ns())
    return last.pg;
  PodGroupPtr found;
  {
    std::shared_lock<std::shared_mutex> g(mu_);
    auto it = pgs_by_key_.find(p.pg_key);
    if (it == pgs_by_key_.end()) return nullptr;
    if (it->second->meta.name == p.pod_group && it->second->meta.ns == p.ns()) found = it->second;
  }
  if (!found) found = pod_group(p.ns(), p.pod_group);  // hash collision: exact lookup
  if (found) last = Last{instance_, p.pg_key, found};
  return found;
}

std::vector<PodGroupPtr> Informers::pod_groups() const {
  std::shared_lock<std::shared_mutex> g(mu_);
  std::vector<PodGroupPtr> out;
  for (const auto& kv : pgs_) out.push_back(kv.second);
  return out;
}

ElasticQuotaPtr Informers::elastic_quota_for_namespace(const std::string& ns) const {
  std::shared_lock<std::shared_mutex> g(mu_);
  auto it = eqs_.lower_bound(ns + "/");
  if (it != eqs_.end() && it->second->meta.ns == ns) return it->second;
  return nullptr;
}

std::vector<ElasticQuotaPtr> Informers::elastic_quotas() const {
  std::shared_lock<std::shared_mutex> g(mu_);
  std::vector<ElasticQuotaPtr> out;
  for (const auto& kv : eqs_) out.push_back(kv.second);
  return out;
}

NRTPtr Informers::nrt(const std::string& node) const {
  std::shared_lock<std::shared_mutex> g(mu_);
  auto it = nrts_.find(node);
  return it == nrts_.end() ? nullptr : it->second;
}

std::vector<PDBPtr> Informers::pdbs() const {
  std::shared_lock<std::shared_mutex> g(mu_);
  std::vector<PDBPtr> out;
  for (const auto& kv : pdbs_) out.push_back(kv.second);
  return out;
}

PriorityClassPtr Informers::priority_class(const std::string& name) const {
  std::shared_lock<std::shared_mutex> g(mu_);
  auto it = pcs_.find(name);
  return it == pcs_.end() ? nullptr : it->second;
}

// ------------------------------------------------------------- storage ----
void Informers::upsert_pv(const PVPtr& pv) {
  std::unique_lock<std::shared_mutex> g(mu_);
  auto it = pvs_.find(pv->meta.name);
  if (it != pvs_.end()) {
    auto& old = pvs_by_class_[it->second->storage_class];
    std::erase(old, it->second);
    it->second = pv;
  } else {
    pvs_.emplace(pv->meta.name, pv);
  }
  pvs_by_class_[pv->storage_class].push_back(pv);
}

void Informers::delete_pv(const std::string& name) {
  std::unique_lock<std::shared_mutex> g(mu_);
  auto it = pvs_.find(name);
  if (it == pvs_.end()) return;
  std::erase(pvs_by_class_[it->second->storage_class], it->second);
  pvs_.erase(it);
}

void Informers::upsert_pvc(const PVCPtr& pvc) {
  std::unique_lock<std::shared_mutex> g(mu_);
  pvcs_[pvc->meta.key()] = pvc;
}

void Informers::delete_pvc(const std::string& key) {
  std::unique_lock<std::shared_mutex> g(mu_);
  pvcs_.erase(key);
}

void Informers::upsert_storage_class(const StorageClassPtr& sc) {
  std::unique_lock<std::shared_mutex> g(mu_);
  scs_[sc->meta.name] = sc;
}

void Informers::delete_storage_class(const std::string& name) {
  std::unique_lock<std::shared_mutex> g(mu_);
  scs_.erase(name);
}

void Informers::upsert_csinode(const CSINodePtr& n) {
  std::unique_lock<std::shared_mutex> g(mu_);
  csinodes_[n->meta.name] = n;
}

void Informers::delete_csinode(const std::string& name) {
  std::unique_lock<std::shared_mutex> g(mu_);
  csinodes_.erase(name);
}

PVPtr Informers::pv(const std::string& name) const {
  std::shared_lock<std::shared_mutex> g(mu_);
  auto it = pvs_.find(name);
  return it == pvs_.end() ? nullptr : it->second;
}

PVCPtr Informers::pvc(const std::string& ns, const std::string& name) const {
  std::shared_lock<std::shared_mutex> g(mu_);
  auto it = pvcs_.find(ns + "/" + name);
  return it == pvcs_.end() ? nullptr : it->second;
}

StorageClassPtr Informers::storage_class(const std::string& name) const {
  std::shared_lock<std::shared_mutex> g(mu_);
  auto it = scs_.find(name);
  return it == scs_.end() ? nullptr : it->second;
}

CSINodePtr Informers::csinode(const std::string& name) const {
  std::shared_lock<std::shared_mutex> g(mu_);
  auto it = csinodes_.find(name);
  return it == csinodes_.end() ? nullptr : it->second;
}

std::vector<PVPtr> Informers::pvs_of_class(const std::string& cls) const {
  std::shared_lock<std::shared_mutex> g(mu_);
  auto it = pvs_by_class_.find(cls);
  return it == pvs_by_class_.end() ? std::vector<PVPtr>{} : it->second;
}

}  // namespace xsched
