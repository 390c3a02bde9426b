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
//     kernarg flush and one doorbell. A run of held packets never wraps the ring end: the packets
//     before the end are committed on their own first (an intercepting queue -- rocprofv3's --
//     hands its handler the run from the write position as ONE array, and a run that wrapped made
//     the handler read past the ring's last page: the round-5 host SIGSEGV);
//   * a cross-lane wait is a barrier-AND packet on the waiting lane, skipped when the signal has
//     already completed;
//   * each lane owns a ring of kSignals completion signals with a use count per slot: a Done is
//     (lane, slot, use), so a Done held long after its slot was reused reads as complete (reuse
//     waits for the previous use's completion), never as the later launch. A slot is reused only
//     after every barrier packet written for its previous use has retired (counted on its lane's
//     retire signal) or, still uncommitted, has had its dependency cleared, so no barrier waits for
//     a later use.
#include "hsa_lane.h"

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <execinfo.h>
#include <fcntl.h>
#include <immintrin.h>
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
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
constexpr int kSignals = 64;           // completion signals of a lane's Done ring
constexpr double kTimeoutUs = 10e6;    // a lane wait longer than this is reported, not spun forever

namespace {

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void queue_error(hsa_status_t s, hsa_queue_t*, void* data);  // records the first error of the lane (data)

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
// EAO_HSA_WRAP_SPLIT=0 lets a committed run of packets wrap the ring end (the round-5 behaviour;
// kept only to reproduce the intercepting-queue fault)
const bool g_wrap_split = [] {
  const char* v = std::getenv("EAO_HSA_WRAP_SPLIT");
  return !(v && v[0] == '0');
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
  std::vector<HsaQueue*> live;  // open HSA lanes (lane_close drops the barrier records naming one)
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

// EAO_SEGV_DIAG=1 (diagnosis only): a host SIGSEGV prints the fault address, the lane commit in
// progress on the faulting thread (ring base / size, the committed run, the read index) and the
// process mappings around the fault address and every return address, then re-raises to the
// previous handler
struct CommitDiag {
  const void* base = nullptr;
  uint64_t size = 0, rd = 0;
  int64_t p0 = -1, p1 = -1;
  int active = 0;
};
thread_local CommitDiag t_commit;
const bool g_segv_diag = [] {
  const char* v = std::getenv("EAO_SEGV_DIAG");
  return v && v[0] == '1';
}();
struct sigaction g_old_segv;

void diag_puts(const char* s) { (void)!write(2, s, std::strlen(s)); }
void diag_hex(const char* k, uint64_t v) {
  char b[64];
  std::snprintf(b, sizeof b, "%s0x%llx", k, (unsigned long long)v);
  diag_puts(b);
}
// the /proc/self/maps lines containing any of the addresses a[0..n)
void diag_maps(const uint64_t* a, int n) {
  const int fd = open("/proc/self/maps", O_RDONLY);
  if (fd < 0) return;
  static char buf[1 << 20];
  size_t len = 0;
  for (ssize_t r; len < sizeof(buf) - 1 && (r = read(fd, buf + len, sizeof(buf) - 1 - len)) > 0;) len += (size_t)r;
  close(fd);
  buf[len] = 0;
  for (char* line = buf; *line;) {
    char* nl = std::strchr(line, '\n');
    if (nl) *nl = 0;
    unsigned long long lo = 0, hi = 0;
    if (std::sscanf(line, "%llx-%llx", &lo, &hi) == 2)
      for (int i = 0; i < n; i++)
        if (a[i] + 0x10000 >= lo && a[i] < hi + 0x10000) {  // the mapping or its neighbours
          diag_puts("  ");
          diag_puts(line);
          diag_puts("\n");
          break;
        }
    if (!nl) break;
    line = nl + 1;
  }
}
void segv_diag(int sig, siginfo_t* si, void* uc) {
  uint64_t a[40];
  a[0] = (uint64_t)si->si_addr;
  void* bt[39];
  const int nb = backtrace(bt, 39);
  for (int i = 0; i < nb; i++) a[1 + i] = (uint64_t)bt[i];
  diag_hex("\n[eao segv diag] fault address ", a[0]);
  if (t_commit.active) {
    diag_hex("\n[eao segv diag] in a lane commit: ring base ", (uint64_t)t_commit.base);
    diag_hex(" size ", t_commit.size);
    diag_hex(" run p0 ", (uint64_t)t_commit.p0);
    diag_hex(" p1 ", (uint64_t)t_commit.p1);
    diag_hex(" read index ", t_commit.rd);
    diag_hex(" ring end ", (uint64_t)t_commit.base + 64 * t_commit.size);
  } else {
    diag_puts("\n[eao segv diag] not in a lane commit");
  }
  diag_puts("\n[eao segv diag] return addresses:");
  for (int i = 0; i < nb; i++) diag_hex(" ", a[1 + i]);
  diag_puts("\n[eao segv diag] mappings:\n");
  diag_maps(a, 1 + nb);
  sigaction(SIGSEGV, &g_old_segv, nullptr);
  (void)sig;
  (void)uc;
}
void segv_diag_install() {
  static bool done = false;
  if (!g_segv_diag || done) return;
  done = true;
  struct sigaction sa {};
  sa.sa_sigaction = segv_diag;
  sa.sa_flags = SA_SIGINFO;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &g_old_segv);
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
  // the A/B switches of the association kernels (assoc.hip, EAO_NP_DIRECT / EAO_NP_SORT256) also
  // reach this code object's own copies of their device variables
  static const struct {
    const char *sym, *env;
    bool flag;
  } kVars[] = {{"_ZN3eao15g_np_direct_maxE", "EAO_NP_DIRECT", false}, {"_ZN3eao12g_np_sort256E", "EAO_NP_SORT256", true}};
  for (const auto& var : kVars) {
    const char* v = std::getenv(var.env);
    if (!v) continue;
    int val = std::atoi(v);
    if (var.flag) val = val != 0;
    hsa_executable_symbol_t sym;
    uint64_t addr = 0;
    s = hsa_executable_get_symbol_by_name(d.exe, var.sym, &d.gpu, &sym);
    if (s == HSA_STATUS_SUCCESS) s = hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_VARIABLE_ADDRESS, &addr);
    if (s == HSA_STATUS_SUCCESS) s = hsa_memory_copy((void*)addr, &val, sizeof(val));
    if (s != HSA_STATUS_SUCCESS) {
      d.why = hsa_msg((std::string("HSA lanes: setting ") + var.env).c_str(), s);
      return &d;
    }
  }
  segv_diag_install();
  d.ok = true;
  return &d;
}

uint16_t header(hsa_packet_type_t t, hsa_fence_scope_t acq, hsa_fence_scope_t rel) {
  return (uint16_t)((t << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                    (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) | (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
}

}  // namespace

// a barrier-AND packet lane_wait wrote on lane q: its packet index, and its ordinal among q's wait
// barriers (their completions count down q's retire signal, in order: the barrier bit)
struct Waiter {
  HsaQueue* q;
  uint64_t idx, k;
};
// a completion signal of a lane's Done ring: its use count, and the barrier-AND packets written
// (on any lane of the same engine) for its current use
struct SigSlot {
  hsa_signal_t s{};
  std::atomic<uint64_t> use{0};
  std::vector<Waiter> waiters;
};
constexpr hsa_signal_value_t kRetire0 = (hsa_signal_value_t)1 << 62;  // a retire signal's initial value

struct HsaQueue {
  hsa_queue_t* q = nullptr;
  unsigned char* karg = nullptr;
  bool karg_dev = false;  // kernargs in device memory (EAO_HSA_KARG=dev)
  DevRt* d = nullptr;
  uint32_t mask = 0;
  std::atomic<int> err{0};  // the lane's first asynchronous queue error (hsa_status_t)
  // packets written but not committed (headers still invalid, doorbell not rung): slots [p0, p1]
  // and their header words; committed together by a record, a sync, a close, or the ring's end
  int64_t p0 = -1, p1 = -1;
  hsa_signal_t sync{};  // lane_sync's completion signal
  // the wait barriers' completion signal: kRetire0 - value = wait barriers completed so far. (The
  // queue's read index cannot tell: under an intercepting queue it counts packets forwarded to the
  // hardware queue, not packets the packet processor has retired.)
  hsa_signal_t retire{};
  uint64_t nwait = 0;      // wait barriers written
  int64_t wait_last = -1;  // index of the latest one (a record must not ride on it)
  std::vector<uint32_t> pword;  // [size]
  const unsigned char* bar_dirty = nullptr;  // last byte written through the BAR (kernargs, inputs), not yet flushed
  SigSlot sigs[kSignals];
  int sig_next = 0;
  int nsig = 0;  // signals created

  void* slot(uint64_t idx) { return (char*)q->base_address + 64 * (idx & mask); }
  bool pending(uint64_t idx) const { return p0 >= 0 && (int64_t)idx >= p0 && (int64_t)idx <= p1; }
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
    if (g_segv_diag) {
      t_commit.base = q->base_address;
      t_commit.size = q->size;
      t_commit.p0 = p0;
      t_commit.p1 = p1;
      t_commit.rd = hsa_queue_load_read_index_relaxed(q);
      t_commit.active = 1;
    }
    flush_kargs();
    for (int64_t i = p0; i <= p1; i++)
      __atomic_store_n((uint32_t*)slot((uint64_t)i), pword[(uint64_t)i & mask], __ATOMIC_RELEASE);
    // the queue's write index moves only here, past complete packets (a tool's intercepting
    // queue reads up to the write index when the doorbell rings)
    hsa_queue_store_write_index_screlease(q, (uint64_t)p1 + 1);
    hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)p1);
    p0 = p1 = -1;
    t_commit.active = 0;
  }
  // a free slot: every packet before the previous one has completed once its successor started
  // (barrier bits), so slots and kernarg slots more than two behind the read index are idle
  uint64_t widx = 0;  // next slot to fill (this lane is the queue's only producer)
  int reserve(uint64_t* out) {
    const uint64_t idx = widx++;
    // the held run ends at the ring's last slot: it goes out on its own, so no committed run wraps
    if ((idx & mask) == 0 && p0 >= 0 && g_wrap_split) commit();
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
  // a barrier-AND packet (pending unless `now`); its index in *at
  int barrier(const hsa_signal_t* dep, int ndep, hsa_signal_t done, bool now, uint64_t* at = nullptr) {
    uint64_t idx;
    if (int rc = reserve(&idx)) return rc;
    hsa_barrier_and_packet_t* p = (hsa_barrier_and_packet_t*)slot(idx);
    std::memset((char*)p + 4, 0, sizeof(*p) - 4);
    for (int i = 0; i < ndep && i < 5; i++) p->dep_signal[i] = dep[i];
    p->completion_signal = done;
    add_pending(idx, header(HSA_PACKET_TYPE_BARRIER_AND, HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_NONE));
    if (at) *at = idx;
    if (now) commit();
    return EAO_OK;
  }
  uint64_t retired() const { return (uint64_t)(kRetire0 - hsa_signal_load_scacquire(retire)); }
  // every barrier packet written for slot k's current use is out of the way: retired by its
  // lane's packet processor, or (still uncommitted, so no packet processor has read it) its
  // dependency cleared -- that use has completed, so the barrier has nothing left to wait for
  int release_waiters(SigSlot& k) {
    for (const Waiter& w : k.waiters) {
      HsaQueue* wq = w.q;
      if (wq->pending(w.idx)) {
        ((hsa_barrier_and_packet_t*)wq->slot(w.idx))->dep_signal[0] = hsa_signal_t{0};
        continue;
      }
      const double t0 = now_us();
      while (wq->retired() < w.k) {
        if (now_us() - t0 > kTimeoutUs) {
          set_error("HSA lane: a wait barrier not retired for 10 s (GPU hung?)");
          return EAO_E_HIP;
        }
        __builtin_ia32_pause();
      }
    }
    k.waiters.clear();
    return EAO_OK;
  }
};

namespace {
void queue_error(hsa_status_t s, hsa_queue_t*, void* data) {
  int z = 0;
  if (data) ((HsaQueue*)data)->err.compare_exchange_strong(z, (int)s);
}
// slot k of d's lane, still on the use d was recorded for (false: reused, so that use completed)
bool same_use(const Done& d) { return d.q->sigs[d.slot].use.load(std::memory_order_acquire) == d.use; }
// d complete: its slot reused since (a reuse waits for the previous use's completion), or the
// signal's value down to 0 while the slot still holds d's use
bool done_complete(const Done& d) {
  if (!same_use(d)) return true;
  const bool zero = hsa_signal_load_scacquire(hsa_signal_t{d.sig}) <= 0;
  return zero || !same_use(d);
}
}  // namespace

bool hsa_lanes_available(int dev) {
  // EAO_HSA_LANES=0: HIP streams (A/B switch). Profiled runs use the lanes too: the host SIGSEGV
  // that rocprofv3's intercepting queue raised (round 5) was a committed run of packets wrapping
  // the ring end, which reserve() no longer lets happen
  static const bool off = [] {
    const char* v = std::getenv("EAO_HSA_LANES");
    return v && v[0] == '0';
  }();
  if (off) return false;
  std::lock_guard<std::mutex> lk(rt().mu);
  return dev_rt(dev)->ok;
}

static void queue_free(HsaQueue* q) {
  for (int i = 0; i < q->nsig; i++) hsa_signal_destroy(q->sigs[i].s);
  if (q->sync.handle) hsa_signal_destroy(q->sync);
  if (q->retire.handle) hsa_signal_destroy(q->retire);
  if (q->karg) hsa_amd_memory_pool_free(q->karg);
  if (q->q) hsa_queue_destroy(q->q);
  delete q;
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
    hsa_status_t s = hsa_queue_create(d->gpu, kQueueSize, HSA_QUEUE_TYPE_SINGLE, queue_error, q, UINT32_MAX,
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
    if (s == HSA_STATUS_SUCCESS) s = hsa_signal_create(0, 0, nullptr, &q->sync);
    if (s == HSA_STATUS_SUCCESS) s = hsa_signal_create(kRetire0, 0, nullptr, &q->retire);
    for (; s == HSA_STATUS_SUCCESS && q->nsig < kSignals; q->nsig++)
      s = hsa_signal_create(0, 0, nullptr, &q->sigs[q->nsig].s);
    if (s != HSA_STATUS_SUCCESS) {
      set_error(hsa_msg("HSA lane: queue", s));
      queue_free(q);
      return EAO_E_HIP;
    }
    q->mask = q->q->size - 1;
    q->pword.assign(q->q->size, 0u);
    q->widx = hsa_queue_load_write_index_relaxed(q->q);
    rt().live.push_back(q);
    l[i].q = q;
  }
  return EAO_OK;
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
    std::lock_guard<std::mutex> lk(rt().mu);
    // barriers on other lanes that wait for this lane's signals retire before the signals
    // go; this lane's own barriers (drained) leave the other lanes' records
    for (SigSlot& k : q->sigs) (void)q->release_waiters(k);
    auto& live = rt().live;
    for (HsaQueue* o : live)
      for (SigSlot& k : o->sigs)
        for (size_t j = 0; j < k.waiters.size();)
          if (k.waiters[j].q == q) {
            k.waiters[j] = k.waiters.back();
            k.waiters.pop_back();
          } else {
            j++;
          }
    for (size_t j = 0; j < live.size(); j++)
      if (live[j] == q) {
        live[j] = live.back();
        live.pop_back();
        break;
      }
    queue_free(q);
  }
  l = Lane();
}

void done_close(Done& d) {
  if (d.e) (void)hipEventDestroy(d.e);
  d = Done();  // ring signals belong to their lane
}

int lane_record(const Lane& l, Done& d) {
  if (!l.q) {
    d.sig = 0;
    d.q = nullptr;
    if (!d.e) EAO_HIP_CHECK(hipEventCreateWithFlags(&d.e, hipEventDisableTiming));
    EAO_HIP_CHECK(hipEventRecord(d.e, l.s));
    return EAO_OK;
  }
  if (d.e) {  // the marker changes kind
    (void)hipEventDestroy(d.e);
    d.e = nullptr;
  }
  HsaQueue* q = l.q;
  const int k = q->sig_next;
  q->sig_next = (k + 1) % kSignals;
  SigSlot& sl = q->sigs[k];
  const double t0 = now_us();
  while (hsa_signal_load_scacquire(sl.s) > 0) {  // its previous use (kSignals records ago) still pending
    if (now_us() - t0 > kTimeoutUs) {
      set_error("HSA lane: completion signal busy for 10 s (GPU hung?)");
      return EAO_E_HIP;
    }
    __builtin_ia32_pause();
  }
  {
    std::lock_guard<std::mutex> lk(rt().mu);
    if (int rc = q->release_waiters(sl)) return rc;
  }
  // the new use: counted before the value rises, so a reader that sees the raised value also
  // sees the new count (done_complete re-reads the count after the value)
  const uint64_t use = sl.use.load(std::memory_order_relaxed) + 1;
  sl.use.store(use, std::memory_order_release);
  hsa_signal_store_screlease(sl.s, 1);
  d.sig = sl.s.handle;
  d.q = q;
  d.slot = (uint32_t)k;
  d.use = use;
  if (q->p1 >= 0 && q->p1 != q->wait_last) {  // ride on the lane's last packet (a dispatch or a barrier-AND: same offset)
    static_assert(offsetof(hsa_kernel_dispatch_packet_t, completion_signal) ==
                      offsetof(hsa_barrier_and_packet_t, completion_signal),
                  "completion signal offset");
    ((hsa_kernel_dispatch_packet_t*)q->slot((uint64_t)q->p1))->completion_signal = sl.s;
    q->commit();
    return EAO_OK;
  }
  return q->barrier(nullptr, 0, sl.s, true);
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
  if (done_complete(d)) return EAO_OK;  // nothing to wait for
  // the barrier is recorded against the use it waits for: that slot's next use waits until the
  // barrier has retired (or clears its dependency while it is still held)
  std::lock_guard<std::mutex> lk(rt().mu);
  const hsa_signal_t s{d.sig};
  uint64_t at = 0;
  if (int rc = l.q->barrier(&s, 1, l.q->retire, false, &at)) return rc;
  l.q->wait_last = (int64_t)at;
  d.q->sigs[d.slot].waiters.push_back(Waiter{l.q, at, ++l.q->nwait});
  return EAO_OK;
}

hipError_t done_query(const Done& d) {
  if (d.e) return hipEventQuery(d.e);
  if (!d.sig) return hipSuccess;
  if (const int e = d.q->err.load(std::memory_order_relaxed)) {
    set_error(hsa_msg("HSA lane: queue error", (hsa_status_t)e));
    return hipErrorLaunchFailure;
  }
  return done_complete(d) ? hipSuccess : hipErrorNotReady;
}

// Self-test of the lanes' completion markers and commits on device `dev` (eao_lane_selftest): three
// HSA lanes, barrier packets only, gates held by host-controlled signals.
//  1. a Done held across 4 kSignals later records of its lane (its slot reused four times) reads
//     complete and needs no barrier; a Done still gated reads not ready, and its slot's reuse waits;
//  2. a barrier written for a gated use but not yet committed when that use completes and its slot
//     is reused: the barrier's dependency is cleared, and the waiting lane drains;
//  3. a committed barrier on a gated use: the slot's reuse waits until the barrier has retired;
//  4. 6000 runs of 1..7 held packets + a record (runs meet the ring end at every alignment),
//     each lane drained.
// Returns 0, or the failing step (> 0) with the message in eao_last_error.
int lane_selftest(int dev, int* report) {
  Lane L[3];
  if (int rc = lanes_open(L, 3, true, dev)) return rc;
  hsa_signal_t gate{};
  int step = 0;
  auto fail = [&](int st, const char* m) {
    set_error(std::string("eao_lane_selftest step ") + std::to_string(st) + ": " + m);
    step = st;
  };
  auto spin = [&](const Done& d) {
    const double t0 = now_us();
    while (done_query(d) == hipErrorNotReady)
      if (now_us() - t0 > 2e6) return false;
    return true;
  };
  auto gated = [&](Lane& l, Done& d) {  // a record on l behind a barrier on the gate
    hsa_signal_store_screlease(gate, 1);
    if (l.q->barrier(&gate, 1, hsa_signal_t{0}, false)) return false;
    return lane_record(l, d) == EAO_OK;
  };
  if (hsa_signal_create(1, 0, nullptr, &gate) != HSA_STATUS_SUCCESS) {
    fail(1, "gate signal");
  }
  Done d0, d1, dx, dy;
  if (!step) {  // 1
    if (!gated(L[0], d0)) fail(1, "gated record");
    else if (done_query(d0) != hipErrorNotReady) fail(1, "a gated Done reads complete");
    hsa_signal_store_screlease(gate, 0);
    if (!step && !spin(d0)) fail(1, "the released Done never completes");
    for (int i = 0; !step && i < 4 * kSignals; i++)
      if (lane_record(L[0], dx)) fail(1, "record");
    if (!step && (done_query(d0) != hipSuccess || d0.q->sigs[d0.slot].use == d0.use))
      fail(1, "the held Done after its slot's reuse");
    const size_t w0 = L[1].q->widx;
    if (!step && (lane_wait(L[1], d0) || L[1].q->widx != w0)) fail(1, "a wait on a completed held Done queued a barrier");
    if (!step && (lane_sync(L[0]) || lane_sync(L[1]))) fail(1, "drain");
  }
  if (!step) {  // 2
    if (!gated(L[0], d1)) fail(2, "gated record");
    else if (lane_wait(L[1], d1)) fail(2, "wait");  // held, uncommitted
    const uint64_t bidx = L[1].q->p1;
    hsa_signal_store_screlease(gate, 0);
    if (!step && !spin(d1)) fail(2, "gated Done");
    for (int i = 0; !step && i < kSignals; i++)  // d1's slot reused: the held barrier is cleared
      if (lane_record(L[0], dx)) fail(2, "record");
    if (!step && (!L[1].q->pending(bidx) ||
                  ((hsa_barrier_and_packet_t*)L[1].q->slot(bidx))->dep_signal[0].handle != 0))
      fail(2, "the held barrier keeps its dependency after the reuse");
    if (!step && (lane_record(L[1], dy) || !spin(dy))) fail(2, "the waiting lane does not drain");
  }
  if (!step) {  // 3
    Done g;
    if (!gated(L[0], g)) fail(3, "gated record");
    else if (lane_wait(L[2], g)) fail(3, "wait");
    const uint64_t k = L[2].q->nwait;  // the barrier on g, committed by the record after it
    if (!step && lane_record(L[2], dy)) fail(3, "record");
    if (!step && L[2].q->retired() >= k) fail(3, "the barrier retired before its gated use");
    hsa_signal_store_screlease(gate, 0);
    for (int i = 0; !step && i < kSignals; i++)
      if (lane_record(L[0], dx)) fail(3, "record");
    if (!step && L[2].q->retired() < k) fail(3, "the slot was reused before the barrier retired");
    if (!step && !spin(dy)) fail(3, "the waiting lane does not drain");
  }
  if (!step) {  // 4
    uint32_t x = 12345;
    for (int it = 0; !step && it < 6000; it++) {
      Lane& l = L[it % 3];
      x = x * 1103515245u + 12345u;
      const int n = 1 + (int)((x >> 16) % 7);
      for (int j = 0; j < n && !step; j++)
        if (l.q->barrier(nullptr, 0, hsa_signal_t{0}, false)) fail(4, "barrier");
      if (!step && lane_record(l, dx)) fail(4, "record");
    }
    for (Lane& l : L)
      if (!step && lane_sync(l)) fail(4, "drain");
    if (report) report[0] = (int)(L[0].q->widx + L[1].q->widx + L[2].q->widx);
  }
  hsa_signal_store_screlease(gate, 0);
  for (Lane& l : L) lane_close(l);
  if (gate.handle) hsa_signal_destroy(gate);
  return step ? EAO_E_STATE : EAO_OK;
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
