// In-process API object store with LIST/WATCH semantics.
//
// Plays the role the reference delegates to kube-apiserver + etcd (the
// integration tests boot a real one through envtest, test/integration/
// main_test.go:31-49). Objects are JSON documents keyed by kind and
// namespace/name; every write bumps a global resourceVersion and fans a watch
// event out to subscribers in commit order. Semantics kept from the apiserver:
//  * create assigns uid / resourceVersion / creationTimestamp, 409 on exists;
//  * update with a stale resourceVersion is a 409 Conflict;
//  * merge-patch (RFC 7386) for PodGroup / ElasticQuota status PATCHes;
//  * pods/binding copies Binding annotations onto the Pod (the behaviour
//    FlexGPU.Bind relies on, pkg/flexgpu/flex_gpu.go:230-242) and 409s when
//    the pod is already bound;
//  * graceful pod deletion sets deletionTimestamp (terminating) first.
// A fault-injection hook (drop/delay/fail per verb+kind) backs the failure
// tests that the reference never had.
#pragma once

#include "common/adaptive_mutex.h"

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "common/json.h"

namespace xsched {

class StoreError : public std::runtime_error {
 public:
  StoreError(int code, const std::string& reason, const std::string& msg)
      : std::runtime_error(msg), code_(code), reason_(reason) {}
  int code() const { return code_; }
  const std::string& reason() const { return reason_; }

 private:
  int code_;
  std::string reason_;
};

enum class EventType : uint8_t { Added, Modified, Deleted, Bookmark };
const char* event_type_name(EventType t);

struct WatchEvent {
  EventType type;
  std::string kind;
  JsonPtr obj;     // new object (or last state for Deleted)
  JsonPtr old;     // previous object for Modified/Deleted (nullptr for Added)
  int64_t rv = 0;
  // A Modified event from a patch that touched only `status` (spec and
  // metadata are those of `old`): a consumer can update its parsed copy of
  // `old` from the status instead of parsing the whole object again.
  bool status_only = false;
};

class Watcher {
 public:
  explicit Watcher(std::set<std::string> kinds, std::string ns) : kinds_(std::move(kinds)), ns_(std::move(ns)) {}
  // Blocks up to timeout_ms for at least one event; returns up to max events.
  std::vector<WatchEvent> next(int timeout_ms, size_t max = 4096);
  void stop();
  bool stopped() const { return stopped_.load(); }
  size_t pending() const;
  bool wants(const std::string& kind, const std::string& ns) const {
    return (kinds_.empty() || kinds_.count(kind)) && (ns_.empty() || ns.empty() || ns == ns_);
  }
  void push(const WatchEvent& ev);
  void push_batch(std::vector<WatchEvent> evs);
  // push / push_batch without the wake-up: true when the consumer is blocked
  // in next() and needs notify(). The store queues events under its own lock
  // this way and wakes consumers after releasing it (a futex wake inside the
  // store's critical section serialised every writer behind it).
  bool push_quiet(const WatchEvent& ev);
  bool push_batch_quiet(std::vector<WatchEvent> evs);
  void notify() { cv_.notify_one(); }

 private:
  std::set<std::string> kinds_;
  std::string ns_;
  mutable AdaptiveMutex mu_;
  std::condition_variable_any cv_;
  std::deque<WatchEvent> q_;
  int waiters_ = 0;  // consumers blocked in next() (guarded by mu_)
  std::atomic<bool> stopped_{false};
};
using WatcherPtr = std::shared_ptr<Watcher>;

struct FaultRule {
  std::string verb;   // create|update|patch|delete|bind|* ...
  std::string kind;   // pods|nodes|...|*
  double fail_prob = 0.0;  // raise 500
  int delay_us = 0;        // sleep before executing
  int remaining = -1;      // -1 = unlimited
};

class ObjectStore {
 public:
  ObjectStore();
  ~ObjectStore();

  JsonPtr create(const std::string& kind, Json obj);
  JsonPtr get(const std::string& kind, const std::string& ns, const std::string& name) const;  // nullptr if absent
  std::vector<JsonPtr> list(const std::string& kind, const std::string& ns, int64_t* rv_out = nullptr) const;
  JsonPtr update(const std::string& kind, Json obj, bool check_rv = true);
  JsonPtr patch(const std::string& kind, const std::string& ns, const std::string& name, const Json& merge_patch);
  // Deletes the object; for pods with grace_seconds > 0 sets deletionTimestamp instead.
  JsonPtr remove(const std::string& kind, const std::string& ns, const std::string& name, int64_t grace_seconds = 0,
                 const std::string& uid_precondition = "");
  JsonPtr bind(const std::string& ns, const std::string& name, const std::string& uid, const std::string& node,
               const Json& annotations);

  // Watch. since_rv > 0 replays retained history after that version (410 Gone
  // if it has been compacted away).
  WatcherPtr watch(const std::set<std::string>& kinds, const std::string& ns = "", int64_t since_rv = 0);
  void unwatch(const WatcherPtr& w);

  int64_t resource_version() const { return rv_.load(); }
  size_t count(const std::string& kind) const;

  void add_fault(const FaultRule& r);
  void clear_faults();

  // Events expire `ttl_us` after creation (kube-apiserver --event-ttl,
  // default 1 h), so a long-running scheduler's FailedScheduling events do not
  // grow the store without bound. Expiry is lazy, on later event writes, and
  // emits DELETED to watchers as etcd's lease expiry does.
  void set_event_ttl_us(int64_t ttl_us);

  // Bulk helpers for benchmarks (one lock hold, one event per object).
  std::vector<JsonPtr> create_many(const std::string& kind, std::vector<Json> objs);
  // Streaming bulk create: `produce` calls emit(obj) per object. Objects are
  // committed in chunks of >= kCreateChunk that end on a PodGroup boundary
  // (pod-group label change), each flushed to watchers as one batch, so a
  // gang is always seen whole while the next chunk is still being produced.
  static constexpr size_t kCreateChunk = 64;
  size_t create_chunked(const std::string& kind,
                        const std::function<void(const std::function<void(Json&&)>&)>& produce);
  size_t delete_all(const std::string& kind, const std::string& ns = "");
  // Deletes the named objects of one namespace under one lock with one watch
  // hand-off (a DeleteCollection by label, e.g. every member of a gang);
  // names not found are skipped. Returns the number deleted.
  size_t remove_many(const std::string& kind, const std::string& ns, const std::vector<std::string>& names);

  static std::string key_of(const std::string& ns, const std::string& name) { return ns.empty() ? name : ns + "/" + name; }
  static bool namespaced(const std::string& kind);

 private:
  struct Entry {
    JsonPtr obj;
  };
  using KindMap = std::unordered_map<std::string, Entry>;

  void check_faults(const std::string& verb, const std::string& kind);
  void expire_events_locked(const std::string& created_key);
  void emit_locked(EventType t, const std::string& kind, const JsonPtr& obj, const JsonPtr& old, int64_t rv,
                   bool status_only = false);
  JsonPtr create_locked(const std::string& kind, Json obj);
  void flush_batch_locked(std::vector<WatchEvent>& batch);
  static void stamp(Json& obj, int64_t rv);
  // Optimistic update of one object: `build(cur)` validates the current
  // version and returns the new object (or nullopt for a no-op) outside the
  // store lock; the result is committed only if the object is still the
  // version `build` saw, else `build` reruns (the deep copy of a Pod no
  // longer happens while 16 binder threads queue on mu_). Returns the
  // committed (or, for a no-op, current) object.
  JsonPtr update_optimistic(const std::string& kind, const std::string& key, const std::string& name,
                            const std::function<std::optional<Json>(const Json& cur)>& build, bool status_only = false);
  std::vector<WatchEvent>* batch_ = nullptr;  // bulk ops collect events here (under mu_)

  // Taken by every writer (16 binder threads, the informer's reads, bulk
  // creates) for short operations: spin before sleeping.
  mutable AdaptiveMutex mu_;
  // Holds mu_ for one store operation. History entries evicted meanwhile
  // are destroyed after the lock is released: the entry is usually the last
  // reference to a deleted object, and freeing its JSON tree under mu_ made
  // every writer (16 binder threads) wait for it once the history was full.
  class Guard {
   public:
    explicit Guard(const ObjectStore& s) : s_(s) { s_.mu_.lock(); }
    ~Guard() {
      std::vector<WatchEvent> dead;
      if (!s_.evicted_.empty()) dead.swap(s_.evicted_);
      std::vector<WatcherPtr> wake;
      if (!s_.wake_.empty()) wake.swap(s_.wake_);
      s_.mu_.unlock();
      for (const auto& w : wake) w->notify();
      if (!dead.empty()) s_.reap(std::move(dead));
    }
    Guard(const Guard&) = delete;
    Guard& operator=(const Guard&) = delete;

   private:
    const ObjectStore& s_;
  };
  mutable std::vector<WatchEvent> evicted_;
  // Watchers that got events under the lock and wait for them (woken by
  // ~Guard, after the unlock).
  mutable std::vector<WatcherPtr> wake_;
  // Evicted entries are freed on a background thread (started on the first
  // eviction), as a garbage-collected API server would: the writer that
  // evicts them does not pay for the JSON trees of objects deleted long ago.
  void reap(std::vector<WatchEvent>&& dead) const;
  void reaper_loop() const;
  mutable std::mutex reap_mu_;
  mutable std::condition_variable reap_cv_;
  mutable std::vector<WatchEvent> reap_q_;
  mutable std::thread reaper_;
  mutable bool reap_stop_ = false;
  void shrink_locked(KindMap& km);
  std::unordered_map<std::string, KindMap> kinds_;
  std::atomic<int64_t> rv_{0};
  std::vector<WatcherPtr> watchers_;
  std::deque<WatchEvent> history_;
  size_t history_cap_ = 50000;
  int64_t event_ttl_us_ = 3600LL * 1000000;
  std::deque<std::pair<int64_t, std::string>> event_expiry_;  // (created wall us, key), creation order
  int64_t compacted_rv_ = 0;
  uint64_t uid_counter_ = 0;
  uint64_t uid_salt_;

  std::mutex fault_mu_;
  std::vector<FaultRule> faults_;
  std::atomic<bool> has_faults_{false};
  std::mt19937_64 fault_rng_{12345};
};

}  // namespace xsched
