// Live MI355X telemetry from the AMD SMI library (libamd_smi, ROCm's
// amd-smi/rocm-smi backend) for the load-watcher provider that feeds
// Trimaran (SURVEY.md §2.9 "Telemetry provider", C19): the reference's
// load-watcher reads CPU/memory from metrics-server/Prometheus/SignalFx
// (vendor/github.com/paypal/load-watcher/pkg/watcher/watcher.go:116-160);
// here each node agent reads its GPUs directly.
//
// Per GPU: GFX and UMC (HBM controller) activity %, per-XCC busy %, VRAM
// used/total, socket power, hotspot/HBM temperature, and the xGMI
// per-link read/write data accumulators (KB) so the caller can turn two
// samples into link throughput. The library is loaded with dlopen at first
// use: the scheduling core does not depend on it, and hosts without AMD GPUs
// (or without the library) report `available() == false` with a reason.
#pragma once

#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

namespace xsched::telemetry {

struct GpuSample {
  int index = 0;          // enumeration order of the library (PCI order)
  std::string bdf;        // dddd:bb:dd.f
  double gfx_activity = -1, umc_activity = -1, mm_activity = -1;  // % (-1 = n/a)
  std::vector<double> xcc_busy;  // instantaneous % per XCC (MI355X: 8)
  int64_t vram_total_mb = -1, vram_used_mb = -1;
  double socket_power_w = -1;
  double temp_hotspot_c = -1, temp_mem_c = -1;
  std::vector<uint64_t> xgmi_read_kb, xgmi_write_kb;  // accumulators per link
  std::vector<int> xgmi_link_up;                       // 1 up, 0 down, -1 n/a
  int xgmi_link_speed = -1, xgmi_link_width = -1;      // as reported by the PMFW table
  int64_t vram_max_bandwidth_gbs = -1;
  uint64_t firmware_timestamp_10ns = 0;  // PMFW clock of this metrics table
  int num_partition = -1;
};

class AmdSmi {
 public:
  static AmdSmi& get();
  bool available();
  const std::string& error() const { return error_; }
  std::vector<GpuSample> sample();

 private:
  AmdSmi() = default;
  bool init_locked();
  std::mutex mu_;
  bool tried_ = false, ok_ = false;
  std::string error_;
  void* lib_ = nullptr;
  std::vector<void*> gpus_;  // amdsmi_processor_handle
};

}  // namespace xsched::telemetry
