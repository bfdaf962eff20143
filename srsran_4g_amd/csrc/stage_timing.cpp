// srsran_4g_amd/csrc/stage_timing.cpp -- per-stage kernel timing with HIP events on the launch
// stream (bench.py reads it to report the dominant kernel's average launch duration live).
#include "stage_timing.h"

#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <vector>

#include "devkey.h"

#include "../../include/srsran_amd_prof.h"

static_assert(srsran_amd::ST_COUNT == SRSRAN_AMD_NOF_STAGES, "stage tables");
static_assert(srsran_amd::HP_COUNT == SRSRAN_AMD_NOF_HOST_PHASES, "host phase tables");

namespace srsran_amd {
namespace {

std::atomic<bool> g_on{false};
std::mutex        g_mu;
struct Rec {
  int        stage;
  int        dev;
  hipEvent_t e0, e1;
};
std::vector<Rec>                       g_pending;
std::map<int, std::vector<hipEvent_t>> g_pool;  // per device: an event is recorded on its own device's streams
double                  g_ms[ST_COUNT];
uint32_t                g_n[ST_COUNT];

hipEvent_t take(int dev)
{
  std::vector<hipEvent_t>& pool = g_pool[dev];
  if (!pool.empty()) {
    hipEvent_t e = pool.back();
    pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  hipEventCreate(&e);
  return e;
}

void drain()  // caller holds g_mu
{
  for (const Rec& r : g_pending) {
    float ms = 0.f;
    if (hipEventSynchronize(r.e1) == hipSuccess && hipEventElapsedTime(&ms, r.e0, r.e1) == hipSuccess) {
      g_ms[r.stage] += ms;
      g_n[r.stage]++;
    }
    g_pool[r.dev].push_back(r.e0);
    g_pool[r.dev].push_back(r.e1);
  }
  g_pending.clear();
}

std::atomic<bool> g_host_on{false};
std::mutex        g_host_mu;
double            g_host_us[HP_COUNT];
uint32_t          g_host_n[HP_COUNT];

int64_t now_ns()
{
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

}  // namespace

HostScope::HostScope(int phase) : phase_(phase)
{
  if (g_host_on.load(std::memory_order_relaxed)) {
    t0_ = now_ns();
  }
}

void HostScope::stop()
{
  if (t0_ < 0) {
    return;
  }
  const double us = (now_ns() - t0_) * 1e-3;
  t0_             = -1;
  std::lock_guard<std::mutex> lk(g_host_mu);
  g_host_us[phase_] += us;
  g_host_n[phase_]++;
}

StageScope::StageScope(int stage, hipStream_t stream) : stage_(stage), stream_(stream)
{
  if (!g_on.load(std::memory_order_relaxed)) {
    return;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  dev_ = cur_dev();
  e0_  = take(dev_);
  if (e0_) {
    hipEventRecord(e0_, stream_);
  }
}

StageScope::~StageScope()
{
  if (!e0_) {
    return;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  hipEvent_t e1 = take(dev_);
  if (!e1) {
    g_pool[dev_].push_back(e0_);
    return;
  }
  hipEventRecord(e1, stream_);
  g_pending.push_back(Rec{stage_, dev_, e0_, e1});
  if (g_pending.size() > 4096) {
    drain();
  }
}

}  // namespace srsran_amd

using namespace srsran_amd;

extern "C" void srsran_amd_timing_enable(int enable)
{
  std::lock_guard<std::mutex> lk(g_mu);
  drain();
  for (int i = 0; i < ST_COUNT; i++) {
    g_ms[i] = 0;
    g_n[i]  = 0;
  }
  g_on.store(enable != 0);
}

extern "C" int srsran_amd_timing_read(float ms[SRSRAN_AMD_NOF_STAGES], uint32_t launches[SRSRAN_AMD_NOF_STAGES])
{
  if (!ms || !launches) {
    return -1;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  drain();
  for (int i = 0; i < ST_COUNT; i++) {
    ms[i]       = (float)g_ms[i];
    launches[i] = g_n[i];
    g_ms[i]     = 0;
    g_n[i]      = 0;
  }
  return 0;
}

extern "C" const char* srsran_amd_stage_name(int stage)
{
  static const char* names[ST_COUNT] = {"ofdm_rx_kernel", "chest_kernel", "predecode_batch_kernel",
                                        "llr_batch_kernel", "rm_rx_lds_kernel", "tdec_kernel", "tb_kernel",
                                        "nr_rm_kernel", "ldpc_kernel", "nr_tb_kernel",
                                        "chest_ul_kernel", "pusch_eq_idft_kernel"};
  return stage >= 0 && stage < ST_COUNT ? names[stage] : "";
}

extern "C" void srsran_amd_host_timing_enable(int enable)
{
  std::lock_guard<std::mutex> lk(g_host_mu);
  for (int i = 0; i < HP_COUNT; i++) {
    g_host_us[i] = 0;
    g_host_n[i]  = 0;
  }
  g_host_on.store(enable != 0);
}

extern "C" int srsran_amd_host_timing_read(double us[SRSRAN_AMD_NOF_HOST_PHASES], uint32_t calls[SRSRAN_AMD_NOF_HOST_PHASES])
{
  if (!us || !calls) {
    return -1;
  }
  std::lock_guard<std::mutex> lk(g_host_mu);
  for (int i = 0; i < HP_COUNT; i++) {
    us[i]        = g_host_us[i];
    calls[i]     = g_host_n[i];
    g_host_us[i] = 0;
    g_host_n[i]  = 0;
  }
  return 0;
}

extern "C" const char* srsran_amd_host_phase_name(int phase)
{
  static const char* names[HP_COUNT] = {"ue_dl_batch", "ofdm_chest_enqueue", "pdsch_descriptors", "pdsch_stage_wait",
                                        "pdsch_launch", "sch_descriptors", "sch_stage_wait", "sch_launch"};
  return phase >= 0 && phase < HP_COUNT ? names[phase] : "";
}
