// cfws_devpolicy.h -- host-only: which device a drop-in frame runs on, and
// the per-device pool of per-thread resources (streams, staging buffers).
//
// coldforce runs every connection on one co_thread's event loop
// (co_event_worker.c:146-183); a multi-thread server hands accepted sockets
// to other threads (co_net_worker.c:240, examples/tcp_server_multi_thread).
// The drop-in therefore keeps its resources per calling thread:
//   * a thread's frames go to the device it was bound to
//     (cfws_bind_thread_device), else to its current HIP device, read on
//     every frame;
//   * when that device changes, the thread hands its resources back to the
//     old device's free list and takes the new device's (or fresh ones);
//   * when the thread exits, its resources go back to the free list, so
//     threads that come and go reuse the same few streams and buffers.
// No HIP types here: cfws_frame.cpp instantiates it with its ThreadDevice,
// tests/test_devpolicy.py with a fake resource (compiled with g++ on CPU).
#pragma once

#include <mutex>
#include <vector>

namespace cfws_policy {

// Res: default-constructible, copyable, with `int device` and `bool holds()
// const` (true when it owns anything worth pooling).
template <class Res, int kMaxDevices>
class DevicePool {
public:
    static constexpr int max_devices = kMaxDevices;

    // A resource for `dev`: the most recently pooled one, or a fresh one
    // (holds() false, device = dev) the caller fills in.
    Res take(int dev)
    {
        if (dev >= 0 && dev < kMaxDevices) {
            std::lock_guard<std::mutex> lock(mu_);
            if (!free_[dev].empty()) {
                Res r = free_[dev].back();
                free_[dev].pop_back();
                return r;
            }
        }
        Res r{};
        r.device = dev;
        return r;
    }

    // Returns r to its device's free list (when it holds anything) and
    // resets r.
    void give(Res& r)
    {
        if (r.device >= 0 && r.device < kMaxDevices && r.holds()) {
            std::lock_guard<std::mutex> lock(mu_);
            free_[r.device].push_back(r);
        }
        r = Res{};
    }

    size_t pooled(int dev)
    {
        if (dev < 0 || dev >= kMaxDevices) return 0;
        std::lock_guard<std::mutex> lock(mu_);
        return free_[dev].size();
    }

private:
    std::mutex mu_;
    std::vector<Res> free_[kMaxDevices];
};

// One per thread (thread_local). Pool& must outlive every thread: the
// library's pool is heap-allocated once and never destroyed.
template <class Res, class Pool>
class ThreadSlot {
public:
    explicit ThreadSlot(Pool& pool) : pool_(pool) {}
    ~ThreadSlot() { pool_.give(res_); }
    ThreadSlot(const ThreadSlot&) = delete;
    ThreadSlot& operator=(const ThreadSlot&) = delete;

    // -1 follows the current device; d >= 0 pins the thread to d.
    bool bind(int dev)
    {
        if (dev < -1 || dev >= Pool::max_devices) return false;
        bound_ = dev;
        return true;
    }
    int bound() const { return bound_; }

    // The device the next frame goes to, given the thread's current device.
    int target(int current) const { return bound_ >= 0 ? bound_ : current; }

    // The thread's resources for `dev`, switching devices when needed.
    Res& on(int dev)
    {
        if (res_.device != dev) {
            pool_.give(res_);
            res_ = pool_.take(dev);
        }
        return res_;
    }

    // Drops the resources without pooling them (the caller freed them).
    void forget() { res_ = Res{}; }
    Res& current() { return res_; }

private:
    Pool& pool_;
    Res res_{};
    int bound_ = -1;
};

}  // namespace cfws_policy
