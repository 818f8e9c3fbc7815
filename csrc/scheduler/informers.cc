#include "scheduler/informers.h"

#include <mutex>

namespace xsched {

namespace {
std::string group_key(const std::string& ns, const std::string& pg) { return ns + "/" + pg; }
}  // namespace

void Informers::upsert_pod(const PodPtr& p) {
  std::unique_lock<std::shared_mutex> g(mu_);
  std::string key = p->key();
  auto it = pods_.find(key);
  if (it != pods_.end() && !it->second->pod_group.empty() && it->second->pod_group != p->pod_group) {
    auto git = pods_by_group_.find(group_key(p->ns(), it->second->pod_group));
    if (git != pods_by_group_.end()) {
      git->second.erase(key);
      if (git->second.empty()) pods_by_group_.erase(git);
    }
  }
  pods_[key] = p;
  if (!p->pod_group.empty()) pods_by_group_[group_key(p->ns(), p->pod_group)].insert(key);
}

void Informers::delete_pod(const Pod& p) {
  std::unique_lock<std::shared_mutex> g(mu_);
  std::string key = p.key();
  auto it = pods_.find(key);
  if (it == pods_.end()) return;
  if (!it->second->pod_group.empty()) {
    auto git = pods_by_group_.find(group_key(p.ns(), it->second->pod_group));
    if (git != pods_by_group_.end()) {
      git->second.erase(key);
      if (git->second.empty()) pods_by_group_.erase(git);
    }
  }
  pods_.erase(it);
}

void Informers::upsert_pod_group(const PodGroupPtr& pg) {
  std::unique_lock<std::shared_mutex> g(mu_);
  pgs_[pg->meta.key()] = pg;
}
void Informers::delete_pod_group(const std::string& key) {
  std::unique_lock<std::shared_mutex> g(mu_);
  pgs_.erase(key);
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
  std::shared_lock<std::shared_mutex> g(mu_);
  auto it = pods_.find(ns + "/" + name);
  return it == pods_.end() ? nullptr : it->second;
}

std::vector<PodPtr> Informers::pods_in_group(const std::string& ns, const std::string& pg) const {
  std::vector<PodPtr> out;
  std::shared_lock<std::shared_mutex> g(mu_);
  auto git = pods_by_group_.find(group_key(ns, pg));
  if (git == pods_by_group_.end()) return out;
  out.reserve(git->second.size());
  for (const auto& k : git->second) {
    auto it = pods_.find(k);
    if (it != pods_.end()) out.push_back(it->second);
  }
  return out;
}

size_t Informers::count_pods_in_group(const std::string& ns, const std::string& pg) const {
  std::shared_lock<std::shared_mutex> g(mu_);
  auto git = pods_by_group_.find(group_key(ns, pg));
  return git == pods_by_group_.end() ? 0 : git->second.size();
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

}  // namespace xsched
