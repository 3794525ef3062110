// host_threads.hpp — a fork-join pool of persistent host threads (the device group's member threads, the pinned
// staging ring's parallel memcpy).  run(f, n): f(0) on the caller's thread, f(1..n-1) on pool threads; returns the
// first non-zero f result in index order.
#pragma once
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

class ForkJoin {
  public:
    explicit ForkJoin(int n) : slots_(n > 0 ? n : 1) {
        for (int i = 1; i < (int)slots_.size(); i++) {
            slots_[i].reset(new Slot());
            Slot* s = slots_[i].get();
            s->th = std::thread([s, i] {
                std::unique_lock<std::mutex> l(s->m);
                for (;;) {
                    s->cv.wait(l, [s] { return s->busy || s->quit; });
                    if (s->quit) return;
                    const std::function<int(int)>* f = s->f;
                    l.unlock();
                    const int rc = (*f)(i);
                    l.lock();
                    s->rc = rc;
                    s->busy = false;
                    s->cv.notify_all();
                }
            });
        }
    }
    ~ForkJoin() {
        for (size_t i = 1; i < slots_.size(); i++) {
            Slot* s = slots_[i].get();
            {
                std::lock_guard<std::mutex> l(s->m);
                s->quit = true;
            }
            s->cv.notify_all();
            s->th.join();
        }
    }
    int size() const { return (int)slots_.size(); }
    // f(i) for every i whose bit is set in `active` (all: ~0), i = 0 on the caller's thread.  One run at a time:
    // a slot holds one f, so concurrent callers serialise here (a second caller overwriting a busy slot's f would
    // make the first caller's f(i) never run while both return as if it had).  f must not call run() itself.
    int run(const std::function<int(int)>& f, uint64_t active = ~0ull) {
        std::lock_guard<std::mutex> one(run_mu_);
        const int n = (int)slots_.size();
        for (int i = 1; i < n; i++) {
            if (!(active >> (i & 63) & 1)) continue;
            Slot* s = slots_[i].get();
            std::lock_guard<std::mutex> l(s->m);
            s->f = &f;
            s->rc = 0;
            s->busy = true;
            s->cv.notify_all();
        }
        int first = (active & 1) ? f(0) : 0;
        for (int i = 1; i < n; i++) {
            if (!(active >> (i & 63) & 1)) continue;
            Slot* s = slots_[i].get();
            std::unique_lock<std::mutex> l(s->m);
            s->cv.wait(l, [s] { return !s->busy; });
            if (!first && s->rc) first = s->rc;
        }
        return first;
    }

  private:
    struct Slot {
        std::thread th;
        std::mutex m;
        std::condition_variable cv;
        const std::function<int(int)>* f = nullptr;
        int rc = 0;
        bool busy = false, quit = false;
    };
    std::vector<std::unique_ptr<Slot>> slots_;
    std::mutex run_mu_;
};
