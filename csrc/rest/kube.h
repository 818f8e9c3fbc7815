// Native service mode against a Kubernetes-style REST API server (ours,
// control/apiserver.py, or kube-apiserver): the scheduler's writes
// (`RestApiClient`) and the LIST/WATCH mirror of the watched kinds into the
// scheduler's local ObjectStore (`RemoteMirror`). Python's RemoteScheduler
// (control/remote.py) wires them when the remote is a REST endpoint.
//
// Reference: the vendored kube-scheduler's client-go informers and its
// binder (vendor/k8s.io/kubernetes/pkg/scheduler/framework/plugins/
// defaultbinder, FlexGPU's Bind at pkg/flexgpu/flex_gpu.go:230-242 posting a
// v1.Binding that carries the GPU index annotation).
#pragma once

#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "framework/plugin.h"
#include "rest/http.h"
#include "store/store.h"

namespace xsched::rest {

// Store kind -> API paths (control/resources.py holds the same table).
struct ResourcePath {
  std::string prefix;  // "/api/v1" or "/apis/<group>/<version>"
  bool namespaced = true;
  std::string api_version, kind;
};
const ResourcePath& resource_path(const std::string& kind);  // throws for unknown kinds
const std::unordered_map<std::string, ResourcePath>& resource_table();
std::string collection_path(const std::string& kind, const std::string& ns);
std::string object_path(const std::string& kind, const std::string& ns, const std::string& name,
                        const std::string& sub = "");

// A pool of keep-alive connections shared by the binder threads.
class ConnPool {
 public:
  explicit ConnPool(Endpoint ep);
  // One request. A pooled connection that turns out to have been closed by
  // the server while idle (EOF or reset before any response byte) is
  // replaced and the request sent once more; `*retried` reports that. A
  // receive timeout or a partial response is never retried: the server may
  // have applied the request (a POST /binding must not be sent twice).
  Response call(const std::string& method, const std::string& path, const std::string& body = "",
                const std::string& content_type = "application/json", bool* retried = nullptr);
  const Endpoint& endpoint() const { return ep_; }
  std::shared_ptr<TlsContext> tls() const { return tls_; }

 private:
  void throttle();  // token bucket (Endpoint::qps / burst)

  Endpoint ep_;
  std::shared_ptr<TlsContext> tls_;
  std::mutex mu_;
  std::vector<std::unique_ptr<HttpConn>> idle_;
  std::mutex rate_mu_;
  double tokens_ = 0;
  int64_t last_refill_ns_ = 0;
};

class RestApiClient : public ApiClient {
 public:
  explicit RestApiClient(Endpoint ep);
  void bind(const Pod& pod, const std::string& node, const Json& annotations) override;
  void delete_pod(const Pod& pod) override;
  void patch(const std::string& kind, const std::string& ns, const std::string& name, const Json& patch) override;
  void record_event(const std::string& kind, const std::string& ns, const std::string& name, const std::string& type,
                    const std::string& reason, const std::string& msg) override;
  uint64_t requests() const { return requests_.load(std::memory_order_relaxed); }

 private:
  ConnPool pool_;
  std::atomic<uint64_t> requests_{0};
};

// LIST + WATCH per kind into a local ObjectStore, one thread per kind:
// ADDED/MODIFIED upsert, DELETED remove, BOOKMARK advances the
// resourceVersion, a server timeout re-watches from it, and an ERROR (410
// Expired) or a failed watch relists, deleting local objects the list no
// longer holds.
class RemoteMirror {
 public:
  RemoteMirror(Endpoint ep, std::shared_ptr<ObjectStore> local, std::vector<std::string> kinds);
  ~RemoteMirror();
  void start();
  bool wait_synced(int timeout_ms);
  void stop();
  uint64_t applied() const { return applied_.load(std::memory_order_relaxed); }
  uint64_t relists() const { return relists_.load(std::memory_order_relaxed); }
  std::string last_error() const;

 private:
  void run(const std::string& kind);
  int64_t relist(const std::string& kind, ConnPool& pool);
  void apply(const std::string& kind, const std::string& type, Json obj);

  Endpoint ep_;
  std::shared_ptr<ObjectStore> local_;
  std::vector<std::string> kinds_;
  std::vector<std::thread> threads_;
  std::atomic<bool> stop_{false};
  mutable std::mutex mu_;
  std::condition_variable synced_cv_;
  size_t synced_ = 0;
  std::vector<HttpConn*> streams_;  // open watch connections (shutdown on stop)
  std::string last_error_;
  std::atomic<uint64_t> applied_{0}, relists_{0};
};

}  // namespace xsched::rest
