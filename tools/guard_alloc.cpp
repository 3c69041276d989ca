// tools/guard_alloc.cpp -- a guard-page device allocator for torch (diagnostics only, never the product).
//
// torch.cuda.memory.CUDAPluggableAllocator(<this .so>, "enf_guard_malloc", "enf_guard_free") replaces
// torch's caching allocator for a test run (tests/conftest.py, ENF_GUARD_ALLOC=1 | 2). Every allocation
// gets its own virtual range [guard | mapped | guard] (hipMemAddressReserve / hipMemCreate / hipMemMap):
//   ENF_GUARD_ALLOC=1: the data END at the end of the mapped pages (rounded up to 16 bytes), so a read or
//                      write past the end of any tensor hits an unmapped page and faults in the kernel
//                      that does it (with torch's caching allocator a small overrun lands in another
//                      block of the same segment and only faults when the segment happens to end there);
//   ENF_GUARD_ALLOC=2: the data START at the mapped start (underruns fault).
// A freed block is unmapped and its physical memory released after its stream is synchronised; the virtual
// range stays reserved, so a later use through a stale pointer faults too. During a stream capture the
// release is deferred to the next free outside a capture.
//   hipcc -O2 -shared -fPIC -o tools/libguard_alloc.so tools/guard_alloc.cpp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

struct Ent {
  void* base;
  size_t total;
  size_t mapped;
  hipMemGenericAllocationHandle_t h;
};

std::mutex mu;
std::unordered_map<void*, Ent> live;
std::vector<Ent> pending;

int mode() {
  static const int m = [] {
    const char* s = std::getenv("ENF_GUARD_ALLOC");
    return s ? std::atoi(s) : 1;
  }();
  return m;
}

void die(const char* what, hipError_t e) {
  std::fprintf(stderr, "enf_guard_alloc: %s failed: %s\n", what, hipGetErrorString(e));
  std::abort();
}

void release(const Ent& e) {
  hipError_t r = hipMemUnmap((char*)e.base + (e.total - e.mapped) / 2, e.mapped);
  if (r != hipSuccess) die("hipMemUnmap", r);
  if ((r = hipMemRelease(e.h)) != hipSuccess) die("hipMemRelease", r);
}

}  // namespace

extern "C" void* enf_guard_malloc(ssize_t size, int device, hipStream_t) {
  std::lock_guard<std::mutex> g(mu);
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = device;
  size_t gran = 0;
  hipError_t r = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum);
  if (r != hipSuccess) die("hipMemGetAllocationGranularity", r);
  const size_t data = ((size_t)(size > 0 ? size : 1) + 15) & ~(size_t)15;
  const size_t mapped = (data + gran - 1) / gran * gran;
  const size_t total = mapped + 2 * gran;
  void* base = nullptr;
  if ((r = hipMemAddressReserve(&base, total, 0, nullptr, 0)) != hipSuccess) die("hipMemAddressReserve", r);
  hipMemGenericAllocationHandle_t h;
  if ((r = hipMemCreate(&h, mapped, &prop, 0)) != hipSuccess) die("hipMemCreate", r);
  char* m0 = (char*)base + gran;
  if ((r = hipMemMap(m0, mapped, 0, h, 0)) != hipSuccess) die("hipMemMap", r);
  hipMemAccessDesc d = {};
  d.location = prop.location;
  d.flags = hipMemAccessFlagsProtReadWrite;
  if ((r = hipMemSetAccess(m0, mapped, &d, 1)) != hipSuccess) die("hipMemSetAccess", r);
  char* p = mode() == 2 ? m0 : m0 + mapped - data;
  live[p] = Ent{base, total, mapped, h};
  return p;
}

extern "C" void enf_guard_free(void* ptr, ssize_t, int, hipStream_t stream) {
  std::lock_guard<std::mutex> g(mu);
  auto it = live.find(ptr);
  if (it == live.end()) return;
  pending.push_back(it->second);
  live.erase(it);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
  if (hipStreamSynchronize(stream) != hipSuccess) return;  // the sticky error is reported elsewhere
  for (const Ent& e : pending) release(e);
  pending.clear();
}
