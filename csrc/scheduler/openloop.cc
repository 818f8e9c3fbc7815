#include "scheduler/openloop.h"

#include <algorithm>
#include <queue>
#include <string>
#include <thread>
#include <unordered_map>

#include "scheduler/scheduler.h"
#include "store/store.h"

namespace xsched {

OpenLoopResult run_open_loop(ObjectStore& store, Scheduler& sched, std::vector<OpenLoopGang> gangs,
                             const std::vector<int64_t>& offsets_us, int64_t hold_us, int64_t timeout_us) {
  const size_t n = std::min(gangs.size(), offsets_us.size());
  OpenLoopResult out;
  out.gangs.resize(n);
  std::unordered_map<std::string, size_t> by_key;  // "ns/pg" -> gang
  std::vector<std::string> ns(n), pg(n);
  std::vector<std::vector<std::string>> members(n);  // pod names, for the deletion
  for (size_t i = 0; i < n; ++i) {
    const Json& md = gangs[i].pod_group["metadata"];
    ns[i] = md["namespace"].str_or("default");
    pg[i] = md["name"].as_string();
    by_key[ns[i] + "/" + pg[i]] = i;
    out.gangs[i].size = static_cast<int>(gangs[i].pods.size());
    for (const auto& p : gangs[i].pods) members[i].push_back(p["metadata"]["name"].as_string());
  }
  (void)sched.gang_records(true);  // start from a clean slate
  using Due = std::pair<int64_t, size_t>;
  std::priority_queue<Due, std::vector<Due>, std::greater<Due>> deletions;
  std::vector<char> deleted(n, 0);
  auto remove_gang = [&](size_t i) {
    if (deleted[i]) return;
    deleted[i] = 1;
    // The gang's members in one call, as `kubectl delete pods -l <group>`.
    try {
      store.remove_many("pods", ns[i], members[i]);
    } catch (const std::exception&) {
    }
    try {
      store.remove("podgroups", ns[i], pg[i]);
    } catch (const std::exception&) {
    }
  };

  auto clock = sched.clock();
  const int64_t t0 = clock->now_us();
  size_t next = 0, done = 0;
  int64_t last_arrival = t0;
  int64_t in_flight = 0, held = 0;
  int64_t next_slice = t0 + 5000;
  Scheduler::Stats st0 = sched.stats();
  uint64_t parks0 = sched.gang_parks();
  for (;;) {
    int64_t now = clock->now_us();
    if (now >= next_slice) {
      const Scheduler::Stats st = sched.stats();
      const uint64_t parks = sched.gang_parks();
      const size_t cache_pods = sched.cache().pod_count(), cache_assumed = sched.cache().assumed_count();
      while (now >= next_slice) {
        out.timeline.push_back({static_cast<int32_t>(in_flight), static_cast<int32_t>(held),
                                static_cast<int32_t>(st.attempts - st0.attempts),
                                static_cast<int32_t>(st.unschedulable - st0.unschedulable),
                                static_cast<int32_t>(parks - parks0), static_cast<int32_t>(cache_pods),
                                static_cast<int32_t>(cache_assumed), static_cast<int32_t>(sched.permit_waiting()),
                                static_cast<int32_t>(sched.bind_backlog())});
        st0 = st;
        parks0 = parks;
        next_slice += 5000;
      }
    }
    bool busy = false;
    // Arrivals due now.
    while (next < n && now >= t0 + offsets_us[next]) {
      out.late_us += now - (t0 + offsets_us[next]);
      OpenLoopGang& g = gangs[next];
      out.gangs[next].create_us = clock->now_us();
      store.create("podgroups", std::move(g.pod_group));
      store.create_many("pods", std::move(g.pods));
      last_arrival = now;
      in_flight += out.gangs[next].size;
      out.max_in_flight_pods = std::max(out.max_in_flight_pods, in_flight);
      ++next;
      busy = true;
      now = clock->now_us();
    }
    // Gangs that completed since the last poll.
    for (const auto& r : sched.gang_records(true)) {
      auto it = by_key.find(r.pg);
      if (it == by_key.end()) continue;
      auto& g = out.gangs[it->second];
      if (g.bound_us) continue;
      g.first_enqueue_us = r.first_enqueue_us;
      g.admit_us = r.admit_us;
      g.bound_us = r.bound_us;
      g.nodes = static_cast<int>(r.nodes.size());
      g.hostable = r.hostable;
      deletions.push({r.bound_us + hold_us, it->second});
      in_flight -= g.size;
      held += g.size;
      out.max_held_pods = std::max(out.max_held_pods, held);
      ++done;
      busy = true;
    }
    // Departures due now.
    while (!deletions.empty() && deletions.top().first <= now) {
      out.delete_late_us += now - deletions.top().first;
      held -= out.gangs[deletions.top().second].size;
      remove_gang(deletions.top().second);
      deletions.pop();
      busy = true;
    }
    if (next == n && (done == n || now - last_arrival > timeout_us)) break;
    if (!busy) {
      int64_t wake = INT64_MAX;
      if (next < n) wake = std::min(wake, t0 + offsets_us[next]);
      if (!deletions.empty()) wake = std::min(wake, deletions.top().first);
      // Completions are polled every ~50 us while gangs are in flight; the
      // recorded timestamps come from the scheduler, so the poll period only
      // delays deletions. Sleeping (not spinning) keeps the driver off the
      // cores the scheduler's threads use.
      if (done < next) wake = std::min(wake, now + 50);
      int64_t d = std::clamp<int64_t>(wake - now, 10, 2000);
      std::this_thread::sleep_for(std::chrono::microseconds(d));
    }
  }
  out.wall_us = clock->now_us() - t0;
  while (!deletions.empty()) {
    remove_gang(deletions.top().second);
    deletions.pop();
  }
  for (size_t i = 0; i < n; ++i) remove_gang(i);
  return out;
}

}  // namespace xsched
