// hsa_lane.cpp -- launch lanes of the association chain (hsa_lane.h): HIP streams, or user-mode
// HSA queues fed with AQL packets written here.
//
// The HSA form loads the association kernels' own gfx950 code object (embedded at build time,
// gen_co.py) into an HSA executable on the GPU agent of the HIP device, and writes the packets
// itself:
//   * a kernel dispatch packet per launch, barrier bit set (in-order, as a stream), acquire at
//     agent scope (device data from kernels on other lanes), release at system scope; the
//     kernel arguments go to a per-slot kernarg ring with the COV5 hidden arguments the kernel
//     declares filled in (grid / block counts, dynamic LDS);
//   * the lane's packets are held uncommitted (headers not yet valid, doorbell not rung) until a
//     Done is recorded on it: the Done rides on the last packet's completion signal instead of an
//     extra barrier packet, and the packets of a forest batch or a frame start go out behind one
//     kernarg flush and one doorbell;
//   * a cross-lane wait is a barrier-AND packet on the waiting lane, skipped when the signal has
//     already completed;
//   * each record takes the next signal of a ring of kSignals, reused only after its previous
//     completion, so a barrier packet still queued on some lane always waits for the use it was
//     written for.
#include "hsa_lane.h"

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <immintrin.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/eao_accel.h"
#include "common.h"

extern "C" const unsigned char eao_assoc_co[], eao_assoc_co_end[];

namespace eao {

static const CoKernel kCo[] = {
#include "assoc_co_meta.inc"
};
constexpr int kNCo = (int)(sizeof(kCo) / sizeof(kCo[0]));
constexpr uint32_t kQueueSize = 1024;  // packets per lane (power of two)
constexpr size_t kKargSlot = 512;      // kernarg bytes per packet slot
constexpr int kSignals = 256;          // completion signals of the Done ring
constexpr double kTimeoutUs = 10e6;    // a lane wait longer than this is reported, not spun forever

namespace {

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

std::atomic<int> g_qerr{0};  // first asynchronous queue error (hsa_status_t)
void queue_error(hsa_status_t s, hsa_queue_t*, void*) {
  int z = 0;
  g_qerr.compare_exchange_strong(z, (int)s);
}

// A/B switches (measurements): EAO_HSA_ACQ = agent (default) | system, the acquire fence of every
// dispatch (at least agent scope: without an acquire fence a kernel can read stale lines of
// reused buffers -- kernarg slots, the batch staging -- from the CUs' caches, a measured GPU
// memory fault); EAO_HSA_KARG = dev (default: device memory written through the BAR, one HDP
// flush + read-back before each doorbell) | host (the CPU's kernarg pool: every wave then loads its
// arguments over PCIe, and the forest's tree kernel takes 10-20 us longer,
// profiles/r05_ab_hsa_kernargs_probe.txt)
const int g_acq = [] {
  const char* v = std::getenv("EAO_HSA_ACQ");
  if (v && v[0] == 's') return (int)HSA_FENCE_SCOPE_SYSTEM;
  return (int)HSA_FENCE_SCOPE_AGENT;
}();
const bool g_dev_karg = [] {
  const char* v = std::getenv("EAO_HSA_KARG");
  return !(v && v[0] == 'h');
}();

struct DevRt {
  bool ok = false;
  std::string why;
  hsa_agent_t gpu{};
  hsa_amd_memory_pool_t dev_pool{};
  bool have_dev_pool = false;
  hsa_amd_hdp_flush_t hdp{};
  hsa_executable_t exe{};
  hsa_code_object_reader_t rd{};
  uint64_t kobj[kNCo] = {};
  hsa_signal_t ring[kSignals] = {};
  int ring_next = 0;
};

struct Rt {
  std::mutex mu;
  bool hsa_up = false;
  std::string why;
  hsa_agent_t cpu{};
  bool have_cpu = false, have_pool = false;
  hsa_amd_memory_pool_t karg_pool{};
  std::vector<hsa_agent_t> gpus;
  std::map<int, DevRt> dev;
};
Rt& rt() {
  static Rt* r = new Rt();  // never destroyed: lanes may close during static teardown
  return *r;
}

hsa_status_t agent_cb(hsa_agent_t a, void* p) {
  Rt* r = (Rt*)p;
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_GPU) r->gpus.push_back(a);
  if (t == HSA_DEVICE_TYPE_CPU && !r->have_cpu) {
    r->cpu = a;
    r->have_cpu = true;
  }
  return HSA_STATUS_SUCCESS;
}
hsa_status_t dev_pool_cb(hsa_amd_memory_pool_t p, void* v) {
  DevRt* d = (DevRt*)v;
  hsa_amd_segment_t seg;
  if (hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  uint32_t fl = 0;
  bool alloc = false;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
  if ((fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && alloc && !d->have_dev_pool) {
    d->dev_pool = p;
    d->have_dev_pool = true;
  }
  return HSA_STATUS_SUCCESS;
}
hsa_status_t pool_cb(hsa_amd_memory_pool_t p, void* v) {
  Rt* r = (Rt*)v;
  hsa_amd_segment_t seg;
  if (hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  uint32_t fl = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
  if ((fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !r->have_pool) {
    r->karg_pool = p;
    r->have_pool = true;
  }
  return HSA_STATUS_SUCCESS;
}

std::string hsa_msg(const char* what, hsa_status_t s) {
  const char* m = nullptr;
  hsa_status_string(s, &m);
  return std::string(what) + ": " + (m ? m : "HSA error");
}

// the process-wide runtime and the code object on `dev`'s agent (under rt().mu)
DevRt* dev_rt(int dev) {
  Rt& r = rt();
  auto it = r.dev.find(dev);
  if (it != r.dev.end()) return &it->second;
  DevRt& d = r.dev[dev];
  if (!r.hsa_up) {
    hsa_status_t s = hsa_init();
    if (s != HSA_STATUS_SUCCESS) {
      d.why = hsa_msg("hsa_init", s);
      return &d;
    }
    r.hsa_up = true;
    hsa_iterate_agents(agent_cb, &r);
    if (r.have_cpu) hsa_amd_agent_iterate_memory_pools(r.cpu, pool_cb, &r);
  }
  if (!r.have_cpu || !r.have_pool) {
    d.why = "HSA lanes: no CPU agent / kernarg pool";
    return &d;
  }
  int bus = -1, devno = -1, dom = -1;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev) != hipSuccess ||
      hipDeviceGetAttribute(&devno, hipDeviceAttributePciDeviceId, dev) != hipSuccess ||
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, dev) != hipSuccess) {
    d.why = "HSA lanes: PCI address of the HIP device unknown";
    return &d;
  }
  bool found = false;
  for (hsa_agent_t g : r.gpus) {
    uint32_t bdf = 0, gdom = 0;
    if (hsa_agent_get_info(g, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS) continue;
    hsa_agent_get_info(g, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &gdom);
    if ((int)((bdf >> 8) & 0xff) == bus && (int)((bdf >> 3) & 0x1f) == devno && (int)gdom == dom) {
      d.gpu = g;
      found = true;
      break;
    }
  }
  if (!found) {
    d.why = "HSA lanes: no HSA agent at the HIP device's PCI address";
    return &d;
  }
  // device memory the host writes through the BAR (kernargs, bar_alloc) and its HDP flush
  hsa_amd_agent_iterate_memory_pools(d.gpu, dev_pool_cb, &d);
  hsa_agent_get_info(d.gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &d.hdp);
  hsa_status_t s = hsa_code_object_reader_create_from_memory(eao_assoc_co, (size_t)(eao_assoc_co_end - eao_assoc_co),
                                                             &d.rd);
  if (s == HSA_STATUS_SUCCESS)
    s = hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &d.exe);
  if (s == HSA_STATUS_SUCCESS) s = hsa_executable_load_agent_code_object(d.exe, d.gpu, d.rd, nullptr, nullptr);
  if (s == HSA_STATUS_SUCCESS) s = hsa_executable_freeze(d.exe, nullptr);
  if (s != HSA_STATUS_SUCCESS) {
    d.why = hsa_msg("HSA lanes: loading the association code object", s);
    return &d;
  }
  for (int k = 0; k < kNCo; k++) {
    hsa_executable_symbol_t sym;
    s = hsa_executable_get_symbol_by_name(d.exe, kCo[k].sym, &d.gpu, &sym);
    uint32_t ks = 0;
    if (s == HSA_STATUS_SUCCESS) s = hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &d.kobj[k]);
    if (s == HSA_STATUS_SUCCESS)
      s = hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &ks);
    if (s != HSA_STATUS_SUCCESS || ks != kCo[k].karg || ks > kKargSlot) {
      d.why = std::string("HSA lanes: kernel ") + kCo[k].name + " missing or not as generated";
      return &d;
    }
  }
  for (int i = 0; i < kSignals; i++)
    if ((s = hsa_signal_create(0, 0, nullptr, &d.ring[i])) != HSA_STATUS_SUCCESS) {
      d.why = hsa_msg("HSA lanes: signals", s);
      return &d;
    }
  d.ok = true;
  return &d;
}

uint16_t header(hsa_packet_type_t t, hsa_fence_scope_t acq, hsa_fence_scope_t rel) {
  return (uint16_t)((t << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                    (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) | (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
}

}  // namespace

struct HsaQueue {
  hsa_queue_t* q = nullptr;
  unsigned char* karg = nullptr;
  bool karg_dev = false;  // kernargs in device memory (EAO_HSA_KARG=dev)
  DevRt* d = nullptr;
  uint32_t mask = 0;
  // packets written but not committed (headers still invalid, doorbell not rung): slots [p0, p1]
  // and their header words; committed together by a record, a sync or a close
  int64_t p0 = -1, p1 = -1;
  hsa_signal_t sync{};  // lane_sync's completion signal
  uint32_t pword[kQueueSize] = {};
  const unsigned char* bar_dirty = nullptr;  // last byte written through the BAR (kernargs, inputs), not yet flushed

  void* slot(uint64_t idx) { return (char*)q->base_address + 64 * (idx & mask); }
  // BAR writes (device-memory kernargs, bar_alloc inputs): out of the write-combining buffer and
  // the HDP before the GPU reads them (the read-back completes only after every earlier posted
  // write has landed)
  void flush_kargs() {
    if (!bar_dirty) return;
    _mm_sfence();
    *(volatile uint32_t*)d->hdp.HDP_MEM_FLUSH_CNTL = 1u;
    (void)*(volatile const unsigned char*)bar_dirty;
    bar_dirty = nullptr;
  }
  void add_pending(uint64_t idx, uint32_t word) {
    if (p0 < 0) p0 = (int64_t)idx;
    p1 = (int64_t)idx;
    pword[idx & mask] = word;
  }
  void commit() {
    if (p0 < 0) return;
    flush_kargs();
    for (int64_t i = p0; i <= p1; i++)
      __atomic_store_n((uint32_t*)slot((uint64_t)i), pword[(uint64_t)i & mask], __ATOMIC_RELEASE);
    // the queue's write index moves only here, past complete packets (a tool's intercepting
    // queue reads up to the write index when the doorbell rings)
    hsa_queue_store_write_index_screlease(q, (uint64_t)p1 + 1);
    hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)p1);
    p0 = p1 = -1;
  }
  // a free slot: every packet before the previous one has completed once its successor started
  // (barrier bits), so slots and kernarg slots more than two behind the read index are idle
  uint64_t widx = 0;  // next slot to fill (this lane is the queue's only producer)
  int reserve(uint64_t* out) {
    const uint64_t idx = widx++;
    const double t0 = now_us();
    while (idx - hsa_queue_load_read_index_scacquire(q) >= (uint64_t)q->size - 2) {
      if (now_us() - t0 > kTimeoutUs) {
        set_error("HSA lane: queue full for 10 s (GPU hung?)");
        return EAO_E_HIP;
      }
      __builtin_ia32_pause();
    }
    __atomic_store_n((uint16_t*)slot(idx), (uint16_t)HSA_PACKET_TYPE_INVALID, __ATOMIC_RELAXED);
    *out = idx;
    return EAO_OK;
  }
  // a barrier-AND packet (pending unless `now`)
  int barrier(const hsa_signal_t* dep, int ndep, hsa_signal_t done, bool now) {
    uint64_t idx;
    if (int rc = reserve(&idx)) return rc;
    hsa_barrier_and_packet_t* p = (hsa_barrier_and_packet_t*)slot(idx);
    std::memset((char*)p + 4, 0, sizeof(*p) - 4);
    for (int i = 0; i < ndep && i < 5; i++) p->dep_signal[i] = dep[i];
    p->completion_signal = done;
    add_pending(idx, header(HSA_PACKET_TYPE_BARRIER_AND, HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_NONE));
    if (now) commit();
    return EAO_OK;
  }
};

bool hsa_lanes_available(int dev) {
  // EAO_HSA_LANES=0: HIP streams; =1: HSA lanes even under a profiler. By default a process
  // profiled by rocprofv3 (its tool library named in ROCP_TOOL_LIBRARIES) uses HIP streams: the
  // tool's queue interception faulted on the host (SIGSEGV inside the doorbell handling, at the
  // first commit on queues created after the process had already run lanes; every run without
  // the tool is clean), so profiles of the association show its HIP-stream form
  static const bool off = [] {
    const char* v = std::getenv("EAO_HSA_LANES");
    if (v) return v[0] == '0';
    return std::getenv("ROCP_TOOL_LIBRARIES") != nullptr;
  }();
  if (off) return false;
  std::lock_guard<std::mutex> lk(rt().mu);
  return dev_rt(dev)->ok;
}

int lanes_open(Lane* l, int n, bool hsa, int dev) {
  for (int i = 0; i < n; i++) l[i] = Lane();
  if (!hsa) {
    int lo = 0, hi = 0;
    EAO_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    for (int i = 0; i < n; i++) EAO_HIP_CHECK(hipStreamCreateWithPriority(&l[i].s, hipStreamNonBlocking, hi));
    return EAO_OK;
  }
  std::lock_guard<std::mutex> lk(rt().mu);
  DevRt* d = dev_rt(dev);
  if (!d->ok) {
    set_error(d->why);
    return EAO_E_HIP;
  }
  for (int i = 0; i < n; i++) {
    HsaQueue* q = new HsaQueue();
    q->d = d;
    hsa_status_t s = hsa_queue_create(d->gpu, kQueueSize, HSA_QUEUE_TYPE_SINGLE, queue_error, nullptr, UINT32_MAX,
                                      UINT32_MAX, &q->q);
    if (s == HSA_STATUS_SUCCESS) hsa_amd_queue_set_priority(q->q, HSA_AMD_QUEUE_PRIORITY_HIGH);
    if (s == HSA_STATUS_SUCCESS && g_dev_karg && d->have_dev_pool && d->hdp.HDP_MEM_FLUSH_CNTL) {
      if (hsa_amd_memory_pool_allocate(d->dev_pool, kKargSlot * q->q->size, 0, (void**)&q->karg) == HSA_STATUS_SUCCESS) {
        if (hsa_amd_agents_allow_access(1, &rt().cpu, nullptr, q->karg) == HSA_STATUS_SUCCESS) {
          q->karg_dev = true;
        } else {
          hsa_amd_memory_pool_free(q->karg);
          q->karg = nullptr;
        }
      }
    }
    if (s == HSA_STATUS_SUCCESS && !q->karg)
      s = hsa_amd_memory_pool_allocate(rt().karg_pool, kKargSlot * q->q->size, 0, (void**)&q->karg);
    if (s == HSA_STATUS_SUCCESS && !q->karg_dev) s = hsa_amd_agents_allow_access(1, &d->gpu, nullptr, q->karg);
    if (s != HSA_STATUS_SUCCESS) {
      set_error(hsa_msg("HSA lane: queue", s));
      if (q->karg) hsa_amd_memory_pool_free(q->karg);
      if (q->q) hsa_queue_destroy(q->q);
      delete q;
      return EAO_E_HIP;
    }
    q->mask = q->q->size - 1;
    q->widx = hsa_queue_load_write_index_relaxed(q->q);
    if (hsa_signal_create(0, 0, nullptr, &q->sync) != HSA_STATUS_SUCCESS) {
      set_error("HSA lane: signal");
      hsa_amd_memory_pool_free(q->karg);
      hsa_queue_destroy(q->q);
      delete q;
      return EAO_E_HIP;
    }
    l[i].q = q;
  }
  return EAO_OK;
}

static hsa_signal_t next_signal(DevRt* d) {
  hsa_signal_t s = d->ring[d->ring_next];
  d->ring_next = (d->ring_next + 1) % kSignals;
  return s;
}

int lane_sync(const Lane& l) {
  if (l.s) EAO_HIP_CHECK(hipStreamSynchronize(l.s));
  if (HsaQueue* q = l.q) {
    // a barrier packet's completion after everything queued, on the lane's own sync signal
    // (created with the lane, destroyed only when it closes: a profiler's interception of the
    // completion may still refer to it after the value has dropped)
    hsa_signal_store_relaxed(q->sync, 1);
    int rc = q->barrier(nullptr, 0, q->sync, true);
    const double t0 = now_us();
    while (rc == EAO_OK && hsa_signal_load_scacquire(q->sync) > 0) {
      if (now_us() - t0 > kTimeoutUs) {
        set_error("HSA lane: not drained after 10 s (GPU hung?)");
        rc = EAO_E_HIP;
      }
      __builtin_ia32_pause();
    }
    return rc;
  }
  return EAO_OK;
}

void lane_close(Lane& l) {
  if (l.s) (void)hipStreamDestroy(l.s);
  if (HsaQueue* q = l.q) {
    Lane t;
    t.q = q;
    (void)lane_sync(t);
    hsa_queue_destroy(q->q);
    hsa_signal_destroy(q->sync);
    hsa_amd_memory_pool_free(q->karg);
    delete q;
  }
  l = Lane();
}

void done_close(Done& d) {
  if (d.e) (void)hipEventDestroy(d.e);
  d = Done();  // ring signals belong to the device runtime
}

int lane_record(const Lane& l, Done& d) {
  if (!l.q) {
    d.sig = 0;
    if (!d.e) EAO_HIP_CHECK(hipEventCreateWithFlags(&d.e, hipEventDisableTiming));
    EAO_HIP_CHECK(hipEventRecord(d.e, l.s));
    return EAO_OK;
  }
  if (d.e) {  // the marker changes kind
    (void)hipEventDestroy(d.e);
    d.e = nullptr;
  }
  HsaQueue* q = l.q;
  hsa_signal_t s;
  {
    std::lock_guard<std::mutex> lk(rt().mu);
    s = next_signal(q->d);
  }
  const double t0 = now_us();
  while (hsa_signal_load_scacquire(s) > 0) {  // its previous use (kSignals records ago) still pending
    if (now_us() - t0 > kTimeoutUs) {
      set_error("HSA lane: completion signal busy for 10 s (GPU hung?)");
      return EAO_E_HIP;
    }
    __builtin_ia32_pause();
  }
  hsa_signal_store_relaxed(s, 1);
  d.sig = s.handle;
  if (q->p1 >= 0) {  // ride on the lane's last packet (a dispatch or a barrier-AND: same offset)
    static_assert(offsetof(hsa_kernel_dispatch_packet_t, completion_signal) ==
                      offsetof(hsa_barrier_and_packet_t, completion_signal),
                  "completion signal offset");
    ((hsa_kernel_dispatch_packet_t*)q->slot((uint64_t)q->p1))->completion_signal = s;
    q->commit();
    return EAO_OK;
  }
  return q->barrier(nullptr, 0, s, true);
}

int lane_wait(const Lane& l, const Done& d) {
  if (!l.q) {
    if (!d.e) {
      set_error("lane_wait: a HIP lane cannot wait on an HSA signal");
      return EAO_E_STATE;
    }
    EAO_HIP_CHECK(hipStreamWaitEvent(l.s, d.e, 0));
    return EAO_OK;
  }
  if (!d.sig) {
    set_error("lane_wait: an HSA lane cannot wait on a HIP event");
    return EAO_E_STATE;
  }
  hsa_signal_t s{d.sig};
  if (hsa_signal_load_relaxed(s) <= 0) return EAO_OK;  // already complete
  return l.q->barrier(&s, 1, hsa_signal_t{0}, false);
}

hipError_t done_query(const Done& d) {
  if (d.e) return hipEventQuery(d.e);
  if (!d.sig) return hipSuccess;
  if (g_qerr.load(std::memory_order_relaxed)) {
    set_error(hsa_msg("HSA lane: queue error", (hsa_status_t)g_qerr.load()));
    return hipErrorLaunchFailure;
  }
  return hsa_signal_load_scacquire(hsa_signal_t{d.sig}) <= 0 ? hipSuccess : hipErrorNotReady;
}

void* bar_alloc(int dev, size_t bytes) {
  std::lock_guard<std::mutex> lk(rt().mu);
  DevRt* d = dev_rt(dev);
  if (!d->ok || !d->have_dev_pool || !d->hdp.HDP_MEM_FLUSH_CNTL) return nullptr;
  void* p = nullptr;
  if (hsa_amd_memory_pool_allocate(d->dev_pool, bytes, 0, &p) != HSA_STATUS_SUCCESS) return nullptr;
  if (hsa_amd_agents_allow_access(1, &rt().cpu, nullptr, p) != HSA_STATUS_SUCCESS) {
    hsa_amd_memory_pool_free(p);
    return nullptr;
  }
  return p;
}
void bar_free(void* p) {
  if (p) hsa_amd_memory_pool_free(p);
}
void lane_bar_written(const Lane& l, const void* last) {
  if (l.q) l.q->bar_dirty = (const unsigned char*)last;
}

int hsa_kernel_id(const char* prefix) {
  const size_t n = std::strlen(prefix);
  for (int k = 0; k < kNCo; k++)
    if (std::strncmp(kCo[k].name, prefix, n) == 0) return k;
  return -1;
}
const CoKernel* hsa_kernel_meta(int id) { return id >= 0 && id < kNCo ? &kCo[id] : nullptr; }

int hsa_arg_mismatch(int id, int i, int size) {
  set_error(std::string("hsa_launch: ") + (id >= 0 && id < kNCo ? kCo[id].name : "unknown kernel") +
            (i < 0 ? ": argument count " : ": argument " + std::to_string(i) + " of size ") + std::to_string(size) +
            " differs from the code object");
  return EAO_E_STATE;
}

int hsa_submit(HsaQueue* q, int id, dim3 g, dim3 b, uint32_t dyn_lds, const unsigned char* args) {
  const CoKernel& k = kCo[id];
  const uint64_t gx = (uint64_t)g.x * b.x, gy = (uint64_t)g.y * b.y, gz = (uint64_t)g.z * b.z;
  if (!g.x || !g.y || !g.z || gx > UINT32_MAX || gy > UINT32_MAX || gz > UINT32_MAX || b.x * b.y * b.z > 1024 ||
      k.group + dyn_lds > 160u * 1024u) {
    set_error(std::string("hsa_launch: launch shape out of range for ") + k.name);
    return EAO_E_ARG;
  }
  // held uncommitted with the lane's other pending packets: the record that follows commits them
  // behind one kernarg flush and one doorbell
  uint64_t idx;
  if (int rc = q->reserve(&idx)) return rc;
  unsigned char* ka = q->karg + kKargSlot * (idx & q->mask);
  std::memcpy(ka, args, k.karg);
  auto put32 = [&](int h, uint32_t v) {
    if (k.hidden[h] >= 0) std::memcpy(ka + k.hidden[h], &v, 4);
  };
  auto put16 = [&](int h, uint16_t v) {
    if (k.hidden[h] >= 0) std::memcpy(ka + k.hidden[h], &v, 2);
  };
  auto put64 = [&](int h, uint64_t v) {
    if (k.hidden[h] >= 0) std::memcpy(ka + k.hidden[h], &v, 8);
  };
  put32(0, g.x), put32(1, g.y), put32(2, g.z);
  put16(3, (uint16_t)b.x), put16(4, (uint16_t)b.y), put16(5, (uint16_t)b.z);
  put16(6, 0), put16(7, 0), put16(8, 0);  // the grid is a whole number of workgroups
  put64(9, 0), put64(10, 0), put64(11, 0);
  put16(12, 3);
  put32(13, dyn_lds);
  if (q->karg_dev) q->bar_dirty = ka + k.karg - 1;
  hsa_kernel_dispatch_packet_t* p = (hsa_kernel_dispatch_packet_t*)q->slot(idx);
  p->workgroup_size_x = (uint16_t)b.x;
  p->workgroup_size_y = (uint16_t)b.y;
  p->workgroup_size_z = (uint16_t)b.z;
  p->reserved0 = 0;
  p->grid_size_x = (uint32_t)gx;
  p->grid_size_y = (uint32_t)gy;
  p->grid_size_z = (uint32_t)gz;
  p->private_segment_size = k.priv;
  p->group_segment_size = k.group + dyn_lds;
  p->kernel_object = q->d->kobj[id];
  p->kernarg_address = ka;
  p->reserved2 = 0;
  p->completion_signal = hsa_signal_t{0};
  q->add_pending(idx, (uint32_t)header(HSA_PACKET_TYPE_KERNEL_DISPATCH, (hsa_fence_scope_t)g_acq,
                                       HSA_FENCE_SCOPE_SYSTEM) |
                          (3u << 16));  // setup: three grid dimensions
  return EAO_OK;
}

}  // namespace eao
