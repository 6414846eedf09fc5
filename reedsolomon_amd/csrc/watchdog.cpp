// watchdog.cpp — see watchdog.hpp.
#include "watchdog.hpp"

#include <pthread.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

namespace rsamd {
namespace detail {

const bool g_watchdog = std::getenv("RSAMD_WATCHDOG") != nullptr;

namespace {
std::mutex g_slots_mu;
std::vector<WatchSlot*> g_slots;  // never freed (threads may exit; their slots stay idle)

uint64_t now_ns() {
    return static_cast<uint64_t>(
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
            .count());
}

void watchdog_loop() {
    for (;;) {
        std::this_thread::sleep_for(std::chrono::milliseconds(500));
        const uint64_t t = now_ns();
        std::lock_guard<std::mutex> lk(g_slots_mu);
        for (WatchSlot* s : g_slots) {
            const char* what = s->what.load(std::memory_order_acquire);
            const uint64_t since = s->since_ns.load(std::memory_order_acquire);
            if (what && t - since > 2000000000ull && !s->told.exchange(true))
                std::fprintf(stderr, "rsamd watchdog: thread %llx inside %s for %.1f s\n",
                             static_cast<unsigned long long>(s->thread.load()), what, (t - since) / 1e9);
        }
    }
}
}  // namespace

WatchSlot* watch_slot() {
    thread_local WatchSlot* mine = nullptr;
    if (mine) return mine;
    mine = new WatchSlot;
    mine->thread.store(static_cast<uint64_t>(pthread_self()));
    std::lock_guard<std::mutex> lk(g_slots_mu);
    if (g_slots.empty()) std::thread(watchdog_loop).detach();
    g_slots.push_back(mine);
    return mine;
}

Region::Region(const char* what) {
    if (!g_watchdog) return;
    slot_ = watch_slot();
    prev_ = slot_->what.load(std::memory_order_relaxed);
    prev_since_ = slot_->since_ns.load(std::memory_order_relaxed);
    slot_->since_ns.store(now_ns(), std::memory_order_release);
    slot_->told.store(false, std::memory_order_relaxed);
    slot_->what.store(what, std::memory_order_release);
}

Region::~Region() {
    if (!slot_) return;
    slot_->what.store(prev_, std::memory_order_release);
    slot_->since_ns.store(prev_since_, std::memory_order_release);
}

}  // namespace detail
}  // namespace rsamd
