#include "store/store.h"

#include "common/clock.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <thread>

#include "api/types.h"

namespace xsched {

const char* event_type_name(EventType t) {
  switch (t) {
    case EventType::Added: return "ADDED";
    case EventType::Modified: return "MODIFIED";
    case EventType::Deleted: return "DELETED";
    case EventType::Bookmark: return "BOOKMARK";
  }
  return "UNKNOWN";
}

// -------------------------------------------------------------- Watcher ----
void Watcher::push(const WatchEvent& ev) {
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    q_.push_back(ev);
  }
  cv_.notify_one();
}

void Watcher::push_batch(std::vector<WatchEvent> evs) {
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    for (auto& e : evs) q_.push_back(std::move(e));
  }
  cv_.notify_one();
}

bool Watcher::push_quiet(const WatchEvent& ev) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  q_.push_back(ev);
  return waiters_ > 0;
}

bool Watcher::push_batch_quiet(std::vector<WatchEvent> evs) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  for (auto& e : evs) q_.push_back(std::move(e));
  return waiters_ > 0;
}

std::vector<WatchEvent> Watcher::next(int timeout_ms, size_t max) {
  std::vector<WatchEvent> out;
  std::unique_lock<AdaptiveMutex> lk(mu_);
  if (q_.empty() && !stopped_.load()) {
    ++waiters_;
    if (timeout_ms < 0)
      cv_.wait(lk, [&] { return !q_.empty() || stopped_.load(); });
    else
      cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return !q_.empty() || stopped_.load(); });
    --waiters_;
  }
  size_t n = std::min(max, q_.size());
  out.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    out.push_back(std::move(q_.front()));
    q_.pop_front();
  }
  return out;
}

void Watcher::stop() {
  {
    std::lock_guard<AdaptiveMutex> g(mu_);  // no lost wake-up against next()
    stopped_.store(true);
  }
  cv_.notify_all();
}

size_t Watcher::pending() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  return q_.size();
}

// ---------------------------------------------------------- ObjectStore ----
ObjectStore::~ObjectStore() {
  {
    std::lock_guard<std::mutex> g(reap_mu_);
    reap_stop_ = true;
  }
  reap_cv_.notify_all();
  if (reaper_.joinable()) reaper_.join();
}

void ObjectStore::reap(std::vector<WatchEvent>&& dead) const {
  {
    std::lock_guard<std::mutex> g(reap_mu_);
    if (reap_stop_) return;  // destroyed here
    if (!reaper_.joinable()) reaper_ = std::thread([this] { reaper_loop(); });
    if (reap_q_.empty()) {
      reap_q_.swap(dead);
    } else {
      for (auto& e : dead) reap_q_.push_back(std::move(e));
    }
  }
  reap_cv_.notify_one();
}

void ObjectStore::reaper_loop() const {
  name_this_thread("xs-reaper");
  std::unique_lock<std::mutex> lk(reap_mu_);
  for (;;) {
    reap_cv_.wait(lk, [&] { return reap_stop_ || !reap_q_.empty(); });
    std::vector<WatchEvent> batch;
    batch.swap(reap_q_);
    lk.unlock();
    batch.clear();  // the frees, off every writer's path
    lk.lock();
    if (reap_stop_ && reap_q_.empty()) return;
  }
}

ObjectStore::ObjectStore() {
  uid_salt_ = static_cast<uint64_t>(std::chrono::steady_clock::now().time_since_epoch().count());
}

bool ObjectStore::namespaced(const std::string& kind) {
  return !(kind == "nodes" || kind == "priorityclasses" || kind == "noderesourcetopologies" || kind == "namespaces" ||
           kind == "loadwatchermetrics" || kind == "persistentvolumes" || kind == "storageclasses" ||
           kind == "csinodes");
}

void ObjectStore::stamp(Json& obj, int64_t rv) {
  obj.at_or_create("metadata").set("resourceVersion", Json(std::to_string(rv)));
}

void ObjectStore::check_faults(const std::string& verb, const std::string& kind) {
  if (!has_faults_.load(std::memory_order_relaxed)) return;
  int delay = 0;
  bool fail = false;
  {
    std::lock_guard<std::mutex> g(fault_mu_);
    for (auto& r : faults_) {
      if (r.remaining == 0) continue;
      if ((r.verb == "*" || r.verb == verb) && (r.kind == "*" || r.kind == kind)) {
        if (r.remaining > 0) --r.remaining;
        delay += r.delay_us;
        if (r.fail_prob > 0.0 && std::uniform_real_distribution<double>(0, 1)(fault_rng_) < r.fail_prob) fail = true;
      }
    }
  }
  if (delay > 0) std::this_thread::sleep_for(std::chrono::microseconds(delay));
  if (fail) throw StoreError(500, "InternalError", "injected fault: " + verb + " " + kind);
}

void ObjectStore::add_fault(const FaultRule& r) {
  std::lock_guard<std::mutex> g(fault_mu_);
  faults_.push_back(r);
  has_faults_.store(true);
}

void ObjectStore::clear_faults() {
  std::lock_guard<std::mutex> g(fault_mu_);
  faults_.clear();
  has_faults_.store(false);
}

void ObjectStore::emit_locked(EventType t, const std::string& kind, const JsonPtr& obj, const JsonPtr& old, int64_t rv,
                              bool status_only) {
  WatchEvent ev{t, kind, obj, old, rv, status_only};
  if (batch_) {
    batch_->push_back(ev);
  } else {
    const Json& md = (*obj)["metadata"];
    const std::string& ns = md["namespace"].as_string();
    for (auto& w : watchers_)
      if (!w->stopped() && w->wants(kind, ns) && w->push_quiet(ev) &&
          std::find(wake_.begin(), wake_.end(), w) == wake_.end())
        wake_.push_back(w);
  }
  history_.push_back(std::move(ev));
  if (history_.size() > history_cap_) {
    compacted_rv_ = history_.front().rv;
    evicted_.push_back(std::move(history_.front()));  // freed by ~Guard, after the lock
    history_.pop_front();
  }
}

JsonPtr ObjectStore::create_locked(const std::string& kind, Json obj) {
  Json& md = obj.at_or_create("metadata");
  std::string name = md["name"].as_string();
  if (name.empty()) {
    std::string gen = md["generateName"].as_string();
    if (gen.empty()) throw StoreError(422, "Invalid", "metadata.name: Required value");
    char buf[16];
    std::snprintf(buf, sizeof buf, "%05llx", static_cast<unsigned long long>((uid_counter_ * 2654435761u) & 0xfffff));
    name = gen + buf;
    md.set("name", Json(name));
  }
  std::string ns = md["namespace"].as_string();
  if (namespaced(kind) && ns.empty()) {
    ns = "default";
    md.set("namespace", Json(ns));
  }
  auto& km = kinds_[kind];
  std::string key = key_of(namespaced(kind) ? ns : "", name);
  if (km.count(key)) throw StoreError(409, "AlreadyExists", kind + " \"" + name + "\" already exists");
  ++uid_counter_;
  char uid[48];
  uint64_t a = uid_counter_ ^ uid_salt_;
  std::snprintf(uid, sizeof uid, "%08llx-%04llx-4%03llx-8%03llx-%012llx",
                static_cast<unsigned long long>(a & 0xffffffff), static_cast<unsigned long long>((a >> 32) & 0xffff),
                static_cast<unsigned long long>((a >> 48) & 0xfff), static_cast<unsigned long long>(uid_counter_ & 0xfff),
                static_cast<unsigned long long>(uid_counter_));
  if (md["uid"].as_string().empty()) md.set("uid", Json(std::string(uid)));
  if (!md["creationTimestamp"].is_string()) md.set("creationTimestamp", Json(format_rfc3339(wall_now_us())));
  if (kind == "pods") {
    Json& st = obj.at_or_create("status");
    if (!st["phase"].is_string()) st.set("phase", Json("Pending"));
  }
  int64_t rv = rv_.fetch_add(1) + 1;
  stamp(obj, rv);
  auto ptr = std::make_shared<const Json>(std::move(obj));
  km[key] = Entry{ptr};
  emit_locked(EventType::Added, kind, ptr, nullptr, rv);
  if (kind == "events") expire_events_locked(key);
  return ptr;
}

void ObjectStore::set_event_ttl_us(int64_t ttl_us) {
  Guard g(*this);
  event_ttl_us_ = ttl_us;
}

void ObjectStore::expire_events_locked(const std::string& created_key) {
  const int64_t now = wall_now_us();
  event_expiry_.emplace_back(now, created_key);
  auto& km = kinds_["events"];
  while (!event_expiry_.empty() && now - event_expiry_.front().first >= event_ttl_us_) {
    auto it = km.find(event_expiry_.front().second);
    event_expiry_.pop_front();
    if (it == km.end()) continue;  // deleted already
    JsonPtr old = it->second.obj;
    km.erase(it);
    emit_locked(EventType::Deleted, "events", old, old, rv_.fetch_add(1) + 1);
  }
}

JsonPtr ObjectStore::create(const std::string& kind, Json obj) {
  check_faults("create", kind);
  Guard g(*this);
  return create_locked(kind, std::move(obj));
}

std::vector<JsonPtr> ObjectStore::create_many(const std::string& kind, std::vector<Json> objs) {
  check_faults("create", kind);
  std::vector<JsonPtr> out;
  out.reserve(objs.size());
  Guard g(*this);
  std::vector<WatchEvent> batch;
  batch_ = &batch;
  try {
    for (auto& o : objs) out.push_back(create_locked(kind, std::move(o)));
  } catch (...) {
    batch_ = nullptr;
    flush_batch_locked(batch);
    throw;
  }
  batch_ = nullptr;
  flush_batch_locked(batch);
  return out;
}

size_t ObjectStore::create_chunked(const std::string& kind,
                                  const std::function<void(const std::function<void(Json&&)>&)>& produce) {
  auto group_of = [](const Json& o) -> const std::string& {
    return o["metadata"]["labels"]["pod-group.scheduling.sigs.k8s.io"].as_string();
  };
  std::vector<Json> chunk;
  chunk.reserve(2 * kCreateChunk);
  size_t n = 0;
  auto flush = [&] {
    if (chunk.empty()) return;
    n += create_many(kind, std::move(chunk)).size();
    chunk.clear();
  };
  produce([&](Json&& o) {
    if (chunk.size() >= kCreateChunk) {
      const std::string& g = group_of(o);
      if (g.empty() || g != group_of(chunk.back())) flush();
    }
    chunk.push_back(std::move(o));
  });
  flush();
  return n;
}

void ObjectStore::flush_batch_locked(std::vector<WatchEvent>& batch) {
  // One hand-off (one lock + one wake-up) per watcher for the whole batch, so
  // an informer sees a bulk create atomically (all PodGroup siblings at once).
  for (auto& w : watchers_) {
    if (w->stopped()) continue;
    std::vector<WatchEvent> mine;
    mine.reserve(batch.size());
    for (const auto& ev : batch) {
      const std::string& ns = (*ev.obj)["metadata"]["namespace"].as_string();
      if (w->wants(ev.kind, ns)) mine.push_back(ev);
    }
    if (!mine.empty() && w->push_batch_quiet(std::move(mine)) && std::find(wake_.begin(), wake_.end(), w) == wake_.end())
      wake_.push_back(w);
  }
}

JsonPtr ObjectStore::get(const std::string& kind, const std::string& ns, const std::string& name) const {
  Guard g(*this);
  auto kit = kinds_.find(kind);
  if (kit == kinds_.end()) return nullptr;
  auto it = kit->second.find(key_of(namespaced(kind) ? ns : "", name));
  return it == kit->second.end() ? nullptr : it->second.obj;
}

std::vector<JsonPtr> ObjectStore::list(const std::string& kind, const std::string& ns, int64_t* rv_out) const {
  std::vector<JsonPtr> out;
  Guard g(*this);
  if (rv_out) *rv_out = rv_.load();
  auto kit = kinds_.find(kind);
  if (kit == kinds_.end()) return out;
  out.reserve(kit->second.size());
  for (const auto& kv : kit->second) {
    if (!ns.empty() && (*kv.second.obj)["metadata"]["namespace"].as_string() != ns) continue;
    out.push_back(kv.second.obj);
  }
  return out;
}

size_t ObjectStore::count(const std::string& kind) const {
  Guard g(*this);
  auto kit = kinds_.find(kind);
  return kit == kinds_.end() ? 0 : kit->second.size();
}

JsonPtr ObjectStore::update(const std::string& kind, Json obj, bool check_rv) {
  check_faults("update", kind);
  Guard g(*this);
  const Json& md = obj["metadata"];
  std::string ns = namespaced(kind) ? md["namespace"].str_or("default") : "";
  std::string name = md["name"].as_string();
  auto& km = kinds_[kind];
  auto it = km.find(key_of(ns, name));
  if (it == km.end()) throw StoreError(404, "NotFound", kind + " \"" + name + "\" not found");
  const Json& cur_md = (*it->second.obj)["metadata"];
  if (check_rv && md["resourceVersion"].is_string() &&
      md["resourceVersion"].as_string() != cur_md["resourceVersion"].as_string())
    throw StoreError(409, "Conflict",
                     "Operation cannot be fulfilled on " + kind + " \"" + name +
                         "\": the object has been modified; please apply your changes to the latest version and try again");
  // Immutable metadata carried over.
  Json& nmd = obj.at_or_create("metadata");
  nmd.set("uid", cur_md["uid"]);
  nmd.set("creationTimestamp", cur_md["creationTimestamp"]);
  if (ns.size()) nmd.set("namespace", Json(ns));
  int64_t rv = rv_.fetch_add(1) + 1;
  stamp(obj, rv);
  auto ptr = std::make_shared<const Json>(std::move(obj));
  JsonPtr old = it->second.obj;
  it->second.obj = ptr;
  emit_locked(EventType::Modified, kind, ptr, old, rv);
  return ptr;
}

JsonPtr ObjectStore::update_optimistic(const std::string& kind, const std::string& key, const std::string& name,
                                       const std::function<std::optional<Json>(const Json& cur)>& build,
                                       bool status_only) {
  for (;;) {
    JsonPtr base;
    {
      Guard g(*this);
      auto& km = kinds_[kind];
      auto it = km.find(key);
      if (it == km.end()) throw StoreError(404, "NotFound", kind + " \"" + name + "\" not found");
      base = it->second.obj;
    }
    std::optional<Json> next = build(*base);  // validation + copy + edit, unlocked
    Guard g(*this);
    auto& km = kinds_[kind];
    auto it = km.find(key);
    if (it == km.end()) throw StoreError(404, "NotFound", kind + " \"" + name + "\" not found");
    if (it->second.obj != base) continue;  // a concurrent write won: rebuild from the new version
    if (!next) return base;
    int64_t rv = rv_.fetch_add(1) + 1;
    stamp(*next, rv);
    auto ptr = std::make_shared<const Json>(std::move(*next));
    it->second.obj = ptr;
    emit_locked(EventType::Modified, kind, ptr, base, rv, status_only);
    return ptr;
  }
}

JsonPtr ObjectStore::patch(const std::string& kind, const std::string& ns, const std::string& name,
                           const Json& merge_patch) {
  check_faults("patch", kind);
  // A patch of `status` alone (plus a resourceVersion precondition) leaves
  // spec and metadata as they were: its event says so (WatchEvent::status_only).
  bool status_only = merge_patch.is_object() && merge_patch.size() > 0;
  for (const auto& [k, v] : merge_patch.members()) {
    if (k == "status") continue;
    if (k == "metadata" && v.is_object() && v.size() == 1 && v.get("resourceVersion")) continue;
    status_only = false;
  }
  return update_optimistic(kind, key_of(namespaced(kind) ? ns : "", name), name,
                           [&](const Json& cur) -> std::optional<Json> {
    // A patch carrying metadata.resourceVersion is a precondition (optimistic
    // concurrency, as kube-apiserver applies it to merge patches).
    if (const Json* pmd = merge_patch.get("metadata")) {
      const Json& prv = (*pmd)["resourceVersion"];
      if (prv.is_string() && !prv.as_string().empty() && prv.as_string() != cur["metadata"]["resourceVersion"].as_string())
        throw StoreError(409, "Conflict",
                         "Operation cannot be fulfilled on " + kind + " \"" + name +
                             "\": the object has been modified; please apply your changes to the latest version and try again");
    }
    Json obj = cur;
    Json saved_md = obj["metadata"];
    obj.merge_patch(merge_patch);
    Json& md = obj.at_or_create("metadata");
    for (const char* k : {"uid", "creationTimestamp", "name", "namespace"})
      if (const Json* v = saved_md.get(k)) md.set(k, *v);
    if (obj == cur) return std::nullopt;  // no-op patch: no new version
    return obj;
  }, status_only);
}

JsonPtr ObjectStore::remove(const std::string& kind, const std::string& ns, const std::string& name,
                            int64_t grace_seconds, const std::string& uid_precondition) {
  check_faults("delete", kind);
  Guard g(*this);
  auto& km = kinds_[kind];
  auto it = km.find(key_of(namespaced(kind) ? ns : "", name));
  if (it == km.end()) throw StoreError(404, "NotFound", kind + " \"" + name + "\" not found");
  if (!uid_precondition.empty() && (*it->second.obj)["metadata"]["uid"].as_string() != uid_precondition)
    throw StoreError(409, "Conflict", "Precondition failed: UID in precondition does not match");
  if (kind == "pods" && grace_seconds > 0) {
    Json obj = *it->second.obj;
    Json& md = obj.at_or_create("metadata");
    if (md["deletionTimestamp"].is_string()) return it->second.obj;  // already terminating
    md.set("deletionTimestamp", Json(format_rfc3339(wall_now_us() + grace_seconds * 1000000)));
    md.set("deletionGracePeriodSeconds", Json(grace_seconds));
    int64_t rv = rv_.fetch_add(1) + 1;
    stamp(obj, rv);
    auto ptr = std::make_shared<const Json>(std::move(obj));
    JsonPtr old = it->second.obj;
    it->second.obj = ptr;
    emit_locked(EventType::Modified, kind, ptr, old, rv);
    return ptr;
  }
  JsonPtr old = it->second.obj;
  km.erase(it);
  shrink_locked(km);
  int64_t rv = rv_.fetch_add(1) + 1;
  emit_locked(EventType::Deleted, kind, old, old, rv);
  return old;
}

// A kind's table keeps the bucket array of its peak size (unordered_map never
// shrinks by itself): after an overload put 10^5 pods in flight, every later
// lookup under the store lock touched a cold, oversized array, and the
// scheduler served ~10% less until a fresh store
// (profiles/r5bc_openloop_fresh_scheduler_same_store.txt). Shrunk once the
// table is 8x emptier than its buckets (amortized O(1) per removal).
void ObjectStore::shrink_locked(KindMap& km) {
  if (km.bucket_count() > 4096 && km.size() * 8 < km.bucket_count()) km.rehash(0);
}

size_t ObjectStore::remove_many(const std::string& kind, const std::string& ns,
                                const std::vector<std::string>& names) {
  check_faults("delete", kind);
  Guard g(*this);
  auto& km = kinds_[kind];
  std::vector<WatchEvent> batch;
  batch_ = &batch;
  size_t n = 0;
  for (const auto& name : names) {
    auto it = km.find(key_of(namespaced(kind) ? ns : "", name));
    if (it == km.end()) continue;
    JsonPtr old = it->second.obj;
    km.erase(it);
    int64_t rv = rv_.fetch_add(1) + 1;
    emit_locked(EventType::Deleted, kind, old, old, rv);
    ++n;
  }
  shrink_locked(km);
  batch_ = nullptr;
  flush_batch_locked(batch);
  return n;
}

size_t ObjectStore::delete_all(const std::string& kind, const std::string& ns) {
  Guard g(*this);
  auto kit = kinds_.find(kind);
  if (kit == kinds_.end()) return 0;
  size_t n = 0;
  std::vector<WatchEvent> batch;
  batch_ = &batch;
  struct Flush {
    ObjectStore* s;
    std::vector<WatchEvent>* b;
    ~Flush() {
      s->batch_ = nullptr;
      s->flush_batch_locked(*b);
    }
  } flush{this, &batch};
  for (auto it = kit->second.begin(); it != kit->second.end();) {
    if (!ns.empty() && (*it->second.obj)["metadata"]["namespace"].as_string() != ns) {
      ++it;
      continue;
    }
    JsonPtr old = it->second.obj;
    it = kit->second.erase(it);
    int64_t rv = rv_.fetch_add(1) + 1;
    emit_locked(EventType::Deleted, kind, old, old, rv);
    ++n;
    // Handed to the watchers in chunks (as kube-apiserver's DeleteCollection
    // deletes item by item): informers start on the first deletions while
    // the rest are still being removed.
    if (batch.size() >= kCreateChunk) {
      flush_batch_locked(batch);
      batch.clear();
    }
  }
  return n;
}

JsonPtr ObjectStore::bind(const std::string& ns, const std::string& name, const std::string& uid,
                          const std::string& node, const Json& annotations) {
  check_faults("bind", "pods");
  const std::string now = format_rfc3339(wall_now_us());
  return update_optimistic("pods", key_of(ns, name), name, [&](const Json& cur) -> std::optional<Json> {
    if (!uid.empty() && cur["metadata"]["uid"].as_string() != uid)
      throw StoreError(409, "Conflict", "Precondition failed: UID in precondition does not match");
    if (!cur["spec"]["nodeName"].as_string().empty())
      throw StoreError(409, "Conflict",
                       "pod " + name + " is already assigned to node \"" + cur["spec"]["nodeName"].as_string() + "\"");
    if (cur["metadata"]["deletionTimestamp"].is_string())
      throw StoreError(409, "Conflict", "pod " + name + " is being deleted, cannot be assigned to a host");
    Json obj = cur;
    obj.at_or_create("spec").set("nodeName", Json(node));
    if (annotations.is_object() && annotations.size()) {
      Json& ann = obj.at_or_create("metadata").at_or_create("annotations");
      for (const auto& kv : annotations.members()) ann.set(kv.first, kv.second);
    }
    Json& st = obj.at_or_create("status");
    Json cond = Json::object();
    cond.set("type", Json("PodScheduled"));
    cond.set("status", Json("True"));
    cond.set("lastTransitionTime", Json(now));
    Json conds = Json::array();
    for (const auto& c : st["conditions"].items())
      if (c["type"].as_string() != "PodScheduled") conds.push_back(c);
    conds.push_back(std::move(cond));
    st.set("conditions", std::move(conds));
    return obj;
  });
}

WatcherPtr ObjectStore::watch(const std::set<std::string>& kinds, const std::string& ns, int64_t since_rv) {
  auto w = std::make_shared<Watcher>(kinds, ns);
  Guard g(*this);
  if (since_rv > 0) {
    if (since_rv < compacted_rv_)
      throw StoreError(410, "Expired", "too old resource version: " + std::to_string(since_rv));
    for (const auto& ev : history_) {
      if (ev.rv <= since_rv) continue;
      const std::string& ens = (*ev.obj)["metadata"]["namespace"].as_string();
      if (w->wants(ev.kind, ens)) w->push(ev);
    }
  }
  watchers_.push_back(w);
  return w;
}

void ObjectStore::unwatch(const WatcherPtr& w) {
  w->stop();
  Guard g(*this);
  for (auto it = watchers_.begin(); it != watchers_.end(); ++it) {
    if (*it == w) {
      watchers_.erase(it);
      break;
    }
  }
}

}  // namespace xsched
