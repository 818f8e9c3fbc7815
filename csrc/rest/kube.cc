#include "rest/kube.h"

#include <algorithm>
#include <chrono>
#include <ctime>
#include <stdexcept>
#include <unordered_map>
#include <unordered_set>

#include "common/clock.h"

namespace xsched::rest {

namespace {

std::string status_message(const Response& r) {
  try {
    Json j = Json::parse(r.body);
    if (j.is_object() && j["message"].is_string()) return j["message"].as_string();
  } catch (const std::exception&) {
  }
  return r.body.substr(0, 200);
}

[[noreturn]] void throw_status(const Response& r, const std::string& what) {
  static const std::unordered_map<int, const char*> kReason = {
      {400, "BadRequest"}, {401, "Unauthorized"}, {403, "Forbidden"}, {404, "NotFound"},
      {409, "Conflict"},   {410, "Expired"},      {422, "Invalid"},   {500, "InternalError"}};
  auto it = kReason.find(r.status);
  throw StoreError(r.status, it == kReason.end() ? "Unknown" : it->second, what + ": " + status_message(r));
}

int64_t rv_of(const Json& obj) {
  const Json& v = obj["metadata"]["resourceVersion"];
  if (v.is_string()) return std::strtoll(v.as_string().c_str(), nullptr, 10);
  return v.as_int(0);
}

}  // namespace

const std::unordered_map<std::string, ResourcePath>& resource_table() {
  static const std::unordered_map<std::string, ResourcePath> kTable = {
      {"pods", {"/api/v1", true, "v1", "Pod"}},
      {"nodes", {"/api/v1", false, "v1", "Node"}},
      {"namespaces", {"/api/v1", false, "v1", "Namespace"}},
      {"events", {"/api/v1", true, "v1", "Event"}},
      {"persistentvolumes", {"/api/v1", false, "v1", "PersistentVolume"}},
      {"persistentvolumeclaims", {"/api/v1", true, "v1", "PersistentVolumeClaim"}},
      {"storageclasses", {"/apis/storage.k8s.io/v1", false, "storage.k8s.io/v1", "StorageClass"}},
      {"csinodes", {"/apis/storage.k8s.io/v1", false, "storage.k8s.io/v1", "CSINode"}},
      {"priorityclasses", {"/apis/scheduling.k8s.io/v1", false, "scheduling.k8s.io/v1", "PriorityClass"}},
      {"poddisruptionbudgets", {"/apis/policy/v1", true, "policy/v1", "PodDisruptionBudget"}},
      {"leases", {"/apis/coordination.k8s.io/v1", true, "coordination.k8s.io/v1", "Lease"}},
      {"podgroups", {"/apis/scheduling.sigs.k8s.io/v1alpha1", true, "scheduling.sigs.k8s.io/v1alpha1", "PodGroup"}},
      {"elasticquotas",
       {"/apis/scheduling.sigs.k8s.io/v1alpha1", true, "scheduling.sigs.k8s.io/v1alpha1", "ElasticQuota"}},
      {"noderesourcetopologies",
       {"/apis/topology.node.k8s.io/v1alpha1", false, "topology.node.k8s.io/v1alpha1", "NodeResourceTopology"}},
      {"loadwatchermetrics", {"/apis/xsched.amd.com/v1alpha1", false, "xsched.amd.com/v1alpha1", "WatcherMetrics"}},
  };
  return kTable;
}

const ResourcePath& resource_path(const std::string& kind) {
  const auto& table = resource_table();
  auto it = table.find(kind);
  if (it == table.end()) throw std::invalid_argument("unknown resource kind " + kind);
  return it->second;
}

std::string collection_path(const std::string& kind, const std::string& ns) {
  const ResourcePath& r = resource_path(kind);
  if (r.namespaced && !ns.empty()) return r.prefix + "/namespaces/" + url_segment(ns) + "/" + kind;
  return r.prefix + "/" + kind;
}

std::string object_path(const std::string& kind, const std::string& ns, const std::string& name,
                        const std::string& sub) {
  const ResourcePath& r = resource_path(kind);
  std::string p = collection_path(kind, r.namespaced ? ns : "") + "/" + url_segment(name);
  if (!sub.empty()) p += "/" + sub;
  return p;
}

// ------------------------------------------------------------ ConnPool ----
ConnPool::ConnPool(Endpoint ep) : ep_(std::move(ep)), tls_(make_tls_context(ep_.tls)) {
  tokens_ = std::max(1, ep_.burst);
}

void ConnPool::throttle() {
  if (ep_.qps <= 0) return;
  const double burst = std::max(1, ep_.burst);
  for (;;) {
    int64_t wait_ns;
    {
      std::lock_guard<std::mutex> g(rate_mu_);
      int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                        std::chrono::steady_clock::now().time_since_epoch()).count();
      if (last_refill_ns_ == 0) last_refill_ns_ = now;
      tokens_ = std::min(burst, tokens_ + static_cast<double>(now - last_refill_ns_) * 1e-9 * ep_.qps);
      last_refill_ns_ = now;
      if (tokens_ >= 1) {
        tokens_ -= 1;
        return;
      }
      wait_ns = static_cast<int64_t>((1 - tokens_) / ep_.qps * 1e9);
    }
    std::this_thread::sleep_for(std::chrono::nanoseconds(wait_ns));
  }
}

Response ConnPool::call(const std::string& method, const std::string& path, const std::string& body,
                        const std::string& content_type, bool* retried) {
  throttle();
  if (retried) *retried = false;
  for (int attempt = 0;; ++attempt) {
    std::unique_ptr<HttpConn> c;
    bool pooled = false;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!idle_.empty()) {
        c = std::move(idle_.back());
        idle_.pop_back();
        pooled = true;
      }
    }
    if (!c) c = std::make_unique<HttpConn>(ep_, tls_);
    try {
      Response r = c->roundtrip(method, path, body, content_type);
      if (c->reusable()) {
        std::lock_guard<std::mutex> g(mu_);
        if (idle_.size() < 64) idle_.push_back(std::move(c));
      }
      return r;
    } catch (const std::runtime_error&) {
      // Only a keep-alive connection the server closed while idle is retried,
      // once, on a fresh connection; anything else (a fresh connection, a
      // timeout, bytes of a response already read) is the caller's error.
      if (!pooled || attempt > 0 || !c->failed_stale()) throw;
      if (retried) *retried = true;
    }
  }
}

// ------------------------------------------------------- RestApiClient ----
RestApiClient::RestApiClient(Endpoint ep) : pool_(std::move(ep)) {}

void RestApiClient::bind(const Pod& pod, const std::string& node, const Json& annotations) {
  Json md = Json::object();
  md.set("name", Json(pod.name()));
  md.set("namespace", Json(pod.ns()));
  if (!pod.uid().empty()) md.set("uid", Json(pod.uid()));
  if (annotations.is_object() && annotations.size() > 0) md.set("annotations", annotations);
  Json target = Json::object();
  target.set("kind", Json("Node"));
  target.set("name", Json(node));
  Json b = Json::object();
  b.set("apiVersion", Json("v1"));
  b.set("kind", Json("Binding"));
  b.set("metadata", std::move(md));
  b.set("target", std::move(target));
  requests_.fetch_add(1, std::memory_order_relaxed);
  bool retried = false;
  Response r = pool_.call("POST", object_path("pods", pod.ns(), pod.name(), "binding"), b.dump(), "application/json",
                          &retried);
  if (r.status == 409 && retried) {
    // The first attempt may have been applied before its connection died:
    // a pod already bound to this very node is this binding's success.
    Response g = pool_.call("GET", object_path("pods", pod.ns(), pod.name()));
    if (g.status == 200) {
      try {
        Json cur = Json::parse(g.body);
        if (cur["spec"]["nodeName"].as_string() == node &&
            (pod.uid().empty() || cur["metadata"]["uid"].as_string() == pod.uid()))
          return;
      } catch (const std::exception&) {
      }
    }
  }
  if (r.status != 200 && r.status != 201) throw_status(r, "binding " + pod.ns() + "/" + pod.name());
}

void RestApiClient::delete_pod(const Pod& pod) {
  Json opts = Json::object();
  opts.set("kind", Json("DeleteOptions"));
  opts.set("apiVersion", Json("v1"));
  opts.set("gracePeriodSeconds", Json(int64_t{0}));
  if (!pod.uid().empty()) {
    Json pre = Json::object();
    pre.set("uid", Json(pod.uid()));
    opts.set("preconditions", std::move(pre));
  }
  requests_.fetch_add(1, std::memory_order_relaxed);
  Response r = pool_.call("DELETE", object_path("pods", pod.ns(), pod.name()), opts.dump());
  if (r.status == 404) return;  // already gone (e.g. preempted twice)
  if (r.status != 200 && r.status != 202) throw_status(r, "deleting " + pod.ns() + "/" + pod.name());
}

void RestApiClient::patch(const std::string& kind, const std::string& ns, const std::string& name, const Json& patch) {
  requests_.fetch_add(1, std::memory_order_relaxed);
  Response r = pool_.call("PATCH", object_path(kind, ns, name), patch.dump(), "application/merge-patch+json");
  if (r.status != 200 && r.status != 201) throw_status(r, "patching " + kind + " " + ns + "/" + name);
}

void RestApiClient::record_event(const std::string& kind, const std::string& ns, const std::string& name,
                                 const std::string& type, const std::string& reason, const std::string& msg) {
  // core/v1 Event, best effort (client-go's recorder never fails its caller).
  std::time_t t = std::time(nullptr);
  char ts[32];
  std::tm tm{};
  gmtime_r(&t, &tm);
  std::strftime(ts, sizeof(ts), "%Y-%m-%dT%H:%M:%SZ", &tm);
  Json md = Json::object();
  md.set("generateName", Json(name + "."));
  md.set("namespace", Json(ns.empty() ? "default" : ns));
  Json ref = Json::object();
  ref.set("kind", Json(kind));
  ref.set("namespace", Json(ns));
  ref.set("name", Json(name));
  Json ev = Json::object();
  ev.set("apiVersion", Json("v1"));
  ev.set("kind", Json("Event"));
  ev.set("metadata", std::move(md));
  ev.set("involvedObject", std::move(ref));
  ev.set("type", Json(type));
  ev.set("reason", Json(reason));
  ev.set("message", Json(msg));
  ev.set("count", Json(int64_t{1}));
  ev.set("firstTimestamp", Json(std::string(ts)));
  ev.set("lastTimestamp", Json(std::string(ts)));
  Json src = Json::object();
  src.set("component", Json("xsched"));
  ev.set("source", std::move(src));
  try {
    requests_.fetch_add(1, std::memory_order_relaxed);
    pool_.call("POST", collection_path("events", ns.empty() ? "default" : ns), ev.dump());
  } catch (const std::exception&) {
  }
}

// -------------------------------------------------------- RemoteMirror ----
RemoteMirror::RemoteMirror(Endpoint ep, std::shared_ptr<ObjectStore> local, std::vector<std::string> kinds)
    : ep_(std::move(ep)), local_(std::move(local)), kinds_(std::move(kinds)) {
  for (const auto& k : kinds_) resource_path(k);  // unknown kinds fail here, not in a thread
}

RemoteMirror::~RemoteMirror() { stop(); }

void RemoteMirror::start() {
  for (const auto& k : kinds_) threads_.emplace_back([this, k] {
    name_this_thread("xs-mirror");
    run(k);
  });
}

bool RemoteMirror::wait_synced(int timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  return synced_cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return synced_ >= kinds_.size(); });
}

void RemoteMirror::stop() {
  if (stop_.exchange(true)) return;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (HttpConn* c : streams_) c->shutdown();
  }
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
}

std::string RemoteMirror::last_error() const {
  std::lock_guard<std::mutex> g(mu_);
  return last_error_;
}

void RemoteMirror::apply(const std::string& kind, const std::string& type, Json obj) {
  const Json& md = obj["metadata"];
  std::string ns = md["namespace"].as_string(), name = md["name"].as_string();
  if (name.empty()) return;
  if (type == "DELETED") {
    try {
      local_->remove(kind, ns, name);
    } catch (const StoreError& e) {
      if (e.code() != 404) throw;
    }
  } else if (local_->get(kind, ns, name)) {
    local_->update(kind, std::move(obj), false);
  } else {
    try {
      local_->create(kind, std::move(obj));
    } catch (const StoreError& e) {
      if (e.code() != 409) throw;
    }
  }
  applied_.fetch_add(1, std::memory_order_relaxed);
}

int64_t RemoteMirror::relist(const std::string& kind, ConnPool& pool) {
  Response r = pool.call("GET", collection_path(kind, ""));
  if (r.status != 200) throw_status(r, "listing " + kind);
  Json list = Json::parse(r.body);
  std::unordered_set<std::string> seen;
  for (const auto& item : list["items"].items()) {
    const Json& md = item["metadata"];
    seen.insert(ObjectStore::key_of(md["namespace"].as_string(), md["name"].as_string()));
    apply(kind, "ADDED", item);
  }
  // Objects deleted while we were not watching.
  for (const auto& obj : local_->list(kind, "")) {
    const Json& md = (*obj)["metadata"];
    std::string key = ObjectStore::key_of(md["namespace"].as_string(), md["name"].as_string());
    if (!seen.count(key)) apply(kind, "DELETED", *obj);
  }
  relists_.fetch_add(1, std::memory_order_relaxed);
  return rv_of(list);
}

void RemoteMirror::run(const std::string& kind) {
  ConnPool pool(ep_);
  bool need_list = true, first = true;
  int64_t rv = 0;
  int failures = 0;
  std::string line;
  auto mark_synced = [&] {
    if (!first) return;
    first = false;
    std::lock_guard<std::mutex> g(mu_);
    ++synced_;
    synced_cv_.notify_all();
  };
  while (!stop_.load()) {
    try {
      if (need_list) {
        try {
          rv = relist(kind, pool);
        } catch (const StoreError& e) {
          if (e.code() != 404) throw;
          // The API does not serve this kind (e.g. a CRD that is not
          // installed): it mirrors as empty, and the list is retried
          // now and then in case the CRD appears.
          {
            std::lock_guard<std::mutex> g(mu_);
            last_error_ = kind + ": " + e.what();
          }
          mark_synced();
          for (int i = 0; i < 300 && !stop_.load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
          continue;
        }
        need_list = false;
        mark_synced();
      }
      HttpConn conn(ep_, pool.tls(), /*streaming=*/true);
      {
        std::lock_guard<std::mutex> g(mu_);
        if (stop_.load()) break;
        streams_.push_back(&conn);
      }
      struct Unregister {
        RemoteMirror* m;
        HttpConn* c;
        ~Unregister() {
          std::lock_guard<std::mutex> g(m->mu_);
          std::erase(m->streams_, c);
        }
      } unregister{this, &conn};
      int status = conn.open_stream(collection_path(kind, "") +
                                    "?watch=true&allowWatchBookmarks=true&timeoutSeconds=300&resourceVersion=" +
                                    std::to_string(rv));
      if (status == 410) {
        need_list = true;
        continue;
      }
      if (status != 200) throw std::runtime_error("watch " + kind + ": HTTP " + std::to_string(status));
      failures = 0;
      while (!stop_.load() && conn.next_line(line)) {
        Json ev = Json::parse(line);
        const std::string& type = ev["type"].as_string();
        if (type == "ERROR") {  // 410 Expired (compacted history) or another failure: relist
          need_list = true;
          break;
        }
        Json* obj = ev.get_mut("object");
        if (!obj) continue;
        if (int64_t v = rv_of(*obj); v > rv) rv = v;
        if (type == "BOOKMARK") continue;
        apply(kind, type, std::move(*obj));
      }
    } catch (const std::exception& e) {
      if (stop_.load()) break;
      {
        std::lock_guard<std::mutex> g(mu_);
        last_error_ = kind + ": " + e.what();
      }
      ++failures;
      if (failures >= 3) need_list = true;
      std::this_thread::sleep_for(std::chrono::milliseconds(std::min(50 * failures, 1000)));
    }
  }
}

}  // namespace xsched::rest
