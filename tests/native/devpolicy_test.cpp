// TEST INFRASTRUCTURE ONLY -- CPU test of the drop-in's device policy and
// per-device resource pool (coldforce_amd/csrc/cfws_devpolicy.h), with a
// fake resource standing in for a stream + staging buffers. Built and run by
// tests/test_devpolicy.py; prints "OK <checks>" or fails with a message.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "cfws_devpolicy.h"

namespace {

std::atomic<int> g_allocs{0};
constexpr int kIds = 4096;
std::atomic<int> g_owner[kIds];    // thread tag holding resource id, 0 = none

struct FakeRes {
    int device = -1;
    int id = 0;                    // 0 = nothing allocated yet
    bool holds() const { return id != 0; }
};

constexpr int kDevs = 8;
using Pool = cfws_policy::DevicePool<FakeRes, kDevs>;
using Slot = cfws_policy::ThreadSlot<FakeRes, Pool>;

Pool& pool()
{
    static Pool* p = new Pool;
    return *p;
}

int checks = 0;
#define CHECK(c)                                                                   \
    do {                                                                           \
        ++checks;                                                                  \
        if (!(c)) {                                                                \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);      \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

// What the drop-in does per frame: pick the device, get the slot's
// resources for it, allocate when fresh.
FakeRes& frame(Slot& s, int current)
{
    FakeRes& r = s.on(s.target(current));
    if (!r.holds()) r.id = ++g_allocs;
    return r;
}

void test_switch_and_bind()
{
    Pool& p = pool();
    Slot s(p);
    FakeRes& a = frame(s, 0);
    const int id0 = a.id;
    CHECK(a.device == 0 && id0 != 0);
    CHECK(frame(s, 0).id == id0);                       // same device: same resources
    FakeRes& b = frame(s, 1);                           // current device moved to 1
    CHECK(b.device == 1 && b.id != id0);
    CHECK(p.pooled(0) == 1);                            // device 0's went back to the pool
    CHECK(frame(s, 0).id == id0);                       // and come back when the thread returns
    CHECK(p.pooled(1) == 1 && p.pooled(0) == 0);
    CHECK(s.bind(3));
    CHECK(frame(s, 0).device == 3);                     // binding overrides the current device
    CHECK(frame(s, 5).device == 3);
    CHECK(s.target(6) == 3);
    CHECK(s.bind(-1));
    CHECK(frame(s, 2).device == 2);                     // unbound: follows the current device again
    CHECK(!s.bind(-2) && !s.bind(kDevs));              // out of range
    CHECK(s.bound() == -1);
}

void test_thread_churn()
{
    // threads that come and go, one after another: each device's resources
    // are allocated once and then reused by every later thread
    const int before = g_allocs.load();
    for (int t = 0; t < 64; ++t) {
        std::thread th([t] {
            Slot s(pool());
            for (int k = 0; k < 10; ++k) frame(s, (t + k) % 4);
        });
        th.join();
    }
    CHECK(g_allocs.load() - before <= 4);
    int pooled = 0;
    for (int d = 0; d < 4; ++d) pooled += (int)pool().pooled(d);
    CHECK(pooled >= 4);
}

void test_concurrent_exclusive()
{
    // 16 threads switching devices at random: a resource is never held by
    // two threads at once, and each ends up back in the pool on exit
    std::vector<std::thread> ths;
    std::atomic<bool> bad{false};
    for (int t = 1; t <= 16; ++t) {
        ths.emplace_back([t, &bad] {
            Slot s(pool());
            std::mt19937 rng(t);
            int held = 0;
            for (int k = 0; k < 20000; ++k) {
                if (rng() % 7 == 0) s.bind((int)(rng() % (kDevs + 1)) - 1);
                const int cur = (int)(rng() % kDevs);
                if (held && s.current().device != s.target(cur)) {
                    g_owner[held % kIds].store(0);   // about to go back to the pool
                    held = 0;
                }
                FakeRes& r = frame(s, cur);
                if (r.id != held) {
                    int expect = 0;
                    if (!g_owner[r.id % kIds].compare_exchange_strong(expect, t)) bad = true;
                    held = r.id;
                }
                if (r.device != s.target(r.device)) bad = true;
            }
            if (held) g_owner[held % kIds].store(0);
        });
    }
    for (auto& th : ths) th.join();
    CHECK(!bad.load());
    CHECK(g_allocs.load() < kIds);
}

}  // namespace

int main()
{
    test_switch_and_bind();
    test_thread_churn();
    test_concurrent_exclusive();
    std::printf("OK %d\n", checks);
    return 0;
}
