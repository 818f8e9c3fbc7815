// Native HTTP API server over the ObjectStore (the envtest / kube-apiserver
// analog for service mode).
//
// The reference runs against a real kube-apiserver (Go) and its integration
// tier boots one through envtest (test/integration/main_test.go:31-49). Our
// first server (control/apiserver.py) is Python's http.server: every request
// pays the interpreter, so a scheduler in another process could bind only
// ~6k pods/s through it (profiles/r2s_remote_bench.jsonl). This one serves
// the same REST surface natively:
//
//   GET    <collection>[?labelSelector=&fieldSelector=&watch=1&resourceVersion=N
//                        &timeoutSeconds=&allowWatchBookmarks=1]
//   POST   <collection>                       create
//   POST   /api/v1/namespaces/<ns>/pods/<name>/binding (annotations copied)
//   GET    <collection>/<name>
//   PUT    <collection>/<name>[/status]       update (resourceVersion precondition)
//   PATCH  <collection>/<name>[/status]       merge / strategic-merge / json-patch
//   DELETE <collection>[/<name>]              DeleteOptions / collection delete
//   GET    /healthz /readyz /livez /version /api /apis
//
// One thread per connection (a scheduler keeps a pool of keep-alive
// connections plus one watch per kind; connections are few and long-lived),
// TCP_NODELAY, responses written in one send. Watches stream chunked JSON
// lines exactly like kube-apiserver (ERROR + 410 Status when the version is
// compacted, BOOKMARKs on request). Bearer-token auth; HTTPS and mutual TLS
// through OpenSSL (the handshake runs on the connection's own thread).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "common/json.h"
#include "store/store.h"

namespace xsched::apiserver {

struct Options {
  std::string host = "127.0.0.1";
  int port = 0;               // 0: pick a free port
  std::string token;          // bearer token ("" = no auth)
  int bookmark_interval_ms = 10'000;
  int max_connections = 4096;
  // HTTPS (kube-apiserver --tls-cert-file / --tls-private-key-file) and,
  // with a client CA, mutual TLS (--client-ca-file). PEM files.
  std::string tls_cert_file, tls_key_file, client_ca_file;
};

// Label / field selector requirement (k8s.io/apimachinery labels + fields
// string syntax: a=b, a==b, a!=b, a in (x,y), a notin (x), a, !a).
struct Requirement {
  enum Op { Eq, Ne, In, NotIn, Exists, NotExists } op = Eq;
  std::string key;
  std::vector<std::string> values;
};
// Throws std::invalid_argument on a malformed selector.
std::vector<Requirement> parse_selector(std::string_view s);
bool labels_match(const std::vector<Requirement>& reqs, const Json& obj);
bool fields_match(const std::vector<Requirement>& reqs, const Json& obj);  // = / != on dotted paths
// RFC 6902 JSON patch; throws std::invalid_argument (HTTP 422) on a bad op.
Json apply_json_patch(const Json& doc, const Json& ops);

class Server {
 public:
  Server(std::shared_ptr<ObjectStore> store, Options o);
  ~Server();
  Server(const Server&) = delete;
  Server& operator=(const Server&) = delete;

  void start();  // binds and starts accepting (throws on bind failure)
  void stop();   // closes the listener, ends every watch and connection, joins
  int port() const { return port_; }
  const std::string& host() const { return opts_.host; }
  uint64_t requests() const { return requests_.load(std::memory_order_relaxed); }
  size_t connections() const;

  struct Request;
  struct Conn;

 private:
  void accept_loop();
  void serve(int fd);
  // Handles one request; false when the connection must close.
  bool handle(Conn& c, Request& r);
  void watch(Conn& c, const std::string& kind, const std::string& ns, Request& r);

  std::shared_ptr<ObjectStore> store_;
  Options opts_;
  void* tls_ctx_ = nullptr;  // SSL_CTX* when serving HTTPS
  int listen_fd_ = -1;
  int port_ = 0;
  std::thread acceptor_;
  std::atomic<bool> stopping_{false};
  std::atomic<uint64_t> requests_{0};
  mutable std::mutex mu_;
  std::condition_variable idle_cv_;
  std::set<int> conns_;                 // open connection fds
  std::set<WatcherPtr> watchers_;       // active watches (stopped on shutdown)
  size_t live_threads_ = 0;
};

}  // namespace xsched::apiserver
