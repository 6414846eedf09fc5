// watchdog.hpp — diagnostics for stalls (env RSAMD_WATCHDOG): code regions
// that may block (HIP runtime calls, engine waits) announce themselves in a
// per-thread slot; a watchdog thread reports every region one thread has
// been inside for more than 2 s, once per entry.  Off by default: a Region
// is then one relaxed load.
#pragma once

#include <atomic>
#include <cstdint>

namespace rsamd {
namespace detail {

struct WatchSlot {
    std::atomic<const char*> what{nullptr};
    std::atomic<uint64_t> since_ns{0};
    std::atomic<uint64_t> thread{0};
    std::atomic<bool> told{false};
};

extern const bool g_watchdog;
WatchSlot* watch_slot();  // this thread's slot (registers it, starts the watchdog once)

class Region {
  public:
    explicit Region(const char* what);
    ~Region();
    Region(const Region&) = delete;
    Region& operator=(const Region&) = delete;

  private:
    WatchSlot* slot_ = nullptr;
    const char* prev_ = nullptr;
    uint64_t prev_since_ = 0;
};

}  // namespace detail
}  // namespace rsamd
