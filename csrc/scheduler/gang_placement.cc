// xGMI gang co-location (gang_placement.h).
#include "scheduler/gang_placement.h"

#include <algorithm>
#include <stdexcept>

#include "scheduler/cache.h"

namespace xsched {

GangPlacement::Mode GangPlacement::parse_mode(const std::string& s) {
  if (s == "Preferred") return Mode::Preferred;
  if (s == "Required") return Mode::Required;
  if (s == "None") return Mode::Off;
  throw std::runtime_error("gangColocation must be Preferred, Required or None, not " + s);
}

const char* GangPlacement::mode_name(Mode m) {
  switch (m) {
    case Mode::Preferred:
      return "Preferred";
    case Mode::Required:
      return "Required";
    default:
      return "None";
  }
}

int64_t GangPlacement::xcd_footprint(int64_t amount, uint8_t mask) {
  int64_t per = 0;
  for (int b = 0; b < 4; ++b) {
    if (!(mask & (1 << b))) continue;
    const int64_t xpp = int64_t{1} << b;
    const int64_t use = (amount + xpp - 1) / xpp * xpp;
    if (per == 0 || use < per) per = use;
  }
  return per;
}

size_t GangPlacement::open_gangs() const {
  std::lock_guard<std::mutex> g(mu_);
  return open_.size();
}

void GangPlacement::reservations_locked(const Snapshot& s, uint64_t self, GpuDemand::Kind kind,
                                        std::vector<std::pair<int, int64_t>>& out) {
  out.clear();
  thread_local std::vector<std::string> hosts;
  for (auto it = open_.begin(); it != open_.end();) {
    const Open& o = it->second;
    if (it->first == self) {
      ++it;
      continue;
    }
    // Only a gang with ranks placed and ranks to go is owed anything; one
    // with none placed (not started, parked, rejected or deleted) is dropped
    // at once and registers again when one of its ranks is planned.
    const int a = cache_->group_placement(it->first, hosts);
    if (a >= o.min_member || a == 0) {
      it = open_.erase(it);
      continue;
    }
    if (o.kind == kind && hosts.size() == 1) {  // anchored: the rest of the gang is owed to that node
      auto ix = s.index.find(hosts[0]);
      if (ix != s.index.end()) {
        const int pos = static_cast<int>(ix->second);
        const int64_t per = kind == GpuDemand::Gpu ? o.amount : xcd_footprint(o.amount, s.part_mask[pos]);
        if (per > 0) out.emplace_back(pos, (o.min_member - a) * per);
      }
    }
    ++it;
  }
}

std::shared_ptr<NodeRestriction> GangPlacement::take_restriction(size_t nodes) {
  // A small ring of restriction objects reused once no cycle holds them (a
  // binding cycle keeps its CycleState, and so the restriction, alive until
  // the bind): no allocation per gang rank in steady state.
  for (size_t k = 0; k < pool_.size(); ++k) {
    auto& r = pool_[(pool_next_ + k) % pool_.size()];
    if (r && r.use_count() == 1) {
      pool_next_ = (pool_next_ + k + 1) % pool_.size();
      r->list.clear();
      r->mask.clear();
      r->nodes = nodes;
      r->fallback = true;
      return r;
    }
  }
  auto r = std::make_shared<NodeRestriction>();
  r->list.reserve(kList);
  r->nodes = nodes;
  if (pool_.size() < kPool) pool_.push_back(r);
  else pool_[pool_next_++ % kPool] = r;
  return r;
}

int GangPlacement::scan(const Snapshot& s, const GpuDemand& d, int64_t members,
                        const std::vector<std::pair<int, int64_t>>& res, std::vector<char>* out_mask,
                        std::vector<int>* out_list) const {
  const int n = static_cast<int>(s.nodes.size());
  if (out_mask) out_mask->assign(static_cast<size_t>(n), 0);
  if (out_list) out_list->clear();
  int count = 0;
  auto take = [&](int pos) {
    ++count;
    if (out_mask) (*out_mask)[static_cast<size_t>(pos)] = 1;
    if (out_list && out_list->size() < kList) out_list->push_back(pos);
  };
  if (d.kind == GpuDemand::Gpu) {
    const int64_t want = members * d.amount;
    const int32_t* fw = s.free_whole.data();
    for (int pos = 0; pos < n; ++pos)
      if (fw[pos] >= want) take(pos);
  } else {
    int64_t want_of[16];
    for (int m = 0; m < 16; ++m) {
      const int64_t per = xcd_footprint(d.amount, static_cast<uint8_t>(m));
      want_of[m] = per > 0 ? members * per : INT64_MAX;
    }
    const int32_t* fx = s.free_xcd.data();
    const uint8_t* pm = s.part_mask.data();
    for (int pos = 0; pos < n; ++pos)
      if (fx[pos] >= want_of[pm[pos] & 15]) take(pos);
  }
  if (res.empty()) return count;
  // Reservations touch few nodes: re-judge those with their owed ranks out.
  std::vector<std::pair<int, int64_t>> owed(res);
  std::sort(owed.begin(), owed.end());
  for (size_t i = 0; i < owed.size();) {
    const int pos = owed[i].first;
    int64_t units = 0;
    for (; i < owed.size() && owed[i].first == pos; ++i) units += owed[i].second;
    const int64_t per =
        d.kind == GpuDemand::Gpu ? d.amount : xcd_footprint(d.amount, s.part_mask[static_cast<size_t>(pos)]);
    const int64_t free = d.kind == GpuDemand::Gpu ? s.free_whole[static_cast<size_t>(pos)]
                                                  : s.free_xcd[static_cast<size_t>(pos)];
    const bool was = per > 0 && free >= members * per;
    const bool now = per > 0 && free - units >= members * per;
    if (was && !now) {
      --count;
      if (out_mask) (*out_mask)[static_cast<size_t>(pos)] = 0;
      if (out_list) out_list->erase(std::remove(out_list->begin(), out_list->end(), pos), out_list->end());
    }
  }
  // A list truncated at kList that lost members is rebuilt from the mask.
  if (out_list && out_mask && count > static_cast<int>(out_list->size()) && out_list->size() < kList) {
    out_list->clear();
    for (int pos = 0; pos < n && out_list->size() < kList; ++pos)
      if ((*out_mask)[static_cast<size_t>(pos)]) out_list->push_back(pos);
  }
  return count;
}

GangPlacement::Plan GangPlacement::plan(const Snapshot& s, const Pod& p, int min_member) {
  Plan out;
  const GpuDemand& d = p.gpu_demand;
  if (mode_ == Mode::Off || !gang_demand(d) || min_member <= 1 || p.pg_key == 0) return out;
  const size_t n = s.nodes.size();
  if (n == 0 || s.free_whole.size() != n || s.free_xcd.size() != n || s.part_mask.size() != n) return out;
  thread_local std::vector<std::string> hosts;
  const int assigned = cache_->group_placement(p.pg_key, hosts);
  out.gang = true;
  out.started = assigned > 0;
  out.remaining = std::max<int64_t>(1, min_member - assigned);
  // Required binds only gangs one node could hold; a larger one spans nodes.
  const bool required = mode_ == Mode::Required && out.remaining <= node_capacity(s, p);
  thread_local std::vector<std::pair<int, int64_t>> res;
  std::lock_guard<std::mutex> g(mu_);
  Open& o = open_[p.pg_key];
  o.kind = d.kind;
  o.amount = d.amount;
  o.min_member = min_member;
  reservations_locked(s, p.pg_key, d.kind, res);
  auto reserved_at = [&](int pos) {
    int64_t u = 0;
    for (const auto& [q, units] : res)
      if (q == pos) u += units;
    return u;
  };
  auto room_at = [&](int pos, int64_t members) {
    const size_t i = static_cast<size_t>(pos);
    const int64_t per = d.kind == GpuDemand::Gpu ? d.amount : xcd_footprint(d.amount, s.part_mask[i]);
    const int64_t free = d.kind == GpuDemand::Gpu ? s.free_whole[i] : s.free_xcd[i];
    return per > 0 && free - reserved_at(pos) >= members * per;
  };
  if (out.started) {
    // Hosts that take every remaining rank, else hosts with room for one
    // more (the gang is split already: fill its nodes first).
    int all_fit[kList], one_fit[kList];
    size_t na = 0, no = 0;
    for (const auto& h : hosts) {
      auto ix = s.index.find(h);
      if (ix == s.index.end()) continue;
      const int pos = static_cast<int>(ix->second);
      if (room_at(pos, out.remaining)) {
        if (na < kList) all_fit[na++] = pos;
      } else if (room_at(pos, 1)) {
        if (no < kList) one_fit[no++] = pos;
      }
    }
    out.hostable = na > 0;
    if (na > 0 || no > 0) {
      auto r = take_restriction(n);
      const int* src = na > 0 ? all_fit : one_fit;
      r->list.assign(src, src + (na > 0 ? na : no));
      std::sort(r->list.begin(), r->list.end());
      // Part of the gang is placed: never strand it (the cycle may still
      // fall back to a node that takes one more rank).
      r->fallback = true;
      out.restriction = std::move(r);
      return out;
    }
  }
  // Nodes that take every remaining rank.
  auto r = take_restriction(n);
  r->fallback = !required;
  const int count = scan(s, d, out.remaining, res, &r->mask, &r->list);
  if (!out.started) out.hostable = count > 0;
  if (count == 0) {
    // Nothing hosts the rest together: Preferred places anyway (split),
    // Required fails the cycle unless the gang is already split.
    if (required && !out.started) {
      r->mask.clear();
      r->list.clear();
      r->fallback = false;
      out.restriction = std::move(r);
    }
    return out;
  }
  if (count == static_cast<int>(n)) return out;  // every node qualifies
  if (static_cast<size_t>(count) <= kList) r->mask.clear();  // the position list is complete
  if (out.started) r->fallback = true;
  out.restriction = std::move(r);
  return out;
}

bool GangPlacement::hostable(const Snapshot& s, const Pod& p, int64_t remaining) {
  const GpuDemand& d = p.gpu_demand;
  const size_t n = s.nodes.size();
  if (!gang_demand(d) || n == 0 || s.free_whole.size() != n) return true;
  thread_local std::vector<std::pair<int, int64_t>> res;
  {
    std::lock_guard<std::mutex> g(mu_);
    reservations_locked(s, p.pg_key, d.kind, res);
  }
  return scan(s, d, std::max<int64_t>(1, remaining), res, nullptr, nullptr) > 0;
}

int64_t GangPlacement::node_capacity(const Snapshot& s, const Pod& p) {
  const GpuDemand& d = p.gpu_demand;
  if (!gang_demand(d)) return 0;
  const uint64_t tag = (static_cast<uint64_t>(d.kind) << 56) ^ static_cast<uint64_t>(d.amount);
  std::lock_guard<std::mutex> g(mu_);
  if (cap_epoch_ != s.node_epoch || cap_nodes_ != s.nodes.size()) {
    cap_memo_.clear();
    cap_epoch_ = s.node_epoch;
    cap_nodes_ = s.nodes.size();
  }
  if (auto it = cap_memo_.find(tag); it != cap_memo_.end()) return it->second;
  int64_t best = 0;
  for (const auto& ni : s.nodes) {
    const GpuLedger& L = ni->gpu;
    int64_t ranks = 0;
    if (d.kind == GpuDemand::Gpu) {
      int64_t spx = 0;
      for (int gi = 0; gi < L.gpu_count; ++gi) spx += L.parts[gi] == 1;
      ranks = spx / d.amount;
    } else {
      for (int gi = 0; gi < L.gpu_count; ++gi) {
        const int xpp = L.xcds_per_part(gi);
        if (xpp <= 0) continue;
        const int64_t use = (d.amount + xpp - 1) / xpp * xpp;
        ranks += 8 / std::max<int64_t>(1, use);
      }
    }
    best = std::max(best, ranks);
  }
  return cap_memo_[tag] = best;
}

}  // namespace xsched
