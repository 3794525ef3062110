// ForkJoin (corda_amd/csrc/host_threads.hpp) under concurrent callers: every caller's f(i) must run for every member
// i, once, before its run() returns (the device group's entries share one pool; ADVICE r05: a second caller used to
// overwrite a busy slot's function, so the first caller's f(i) never ran while both returned success).
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>
#include "host_threads.hpp"

int main() {
    const int members = 4, callers = 6, calls = 3000;
    ForkJoin pool(members);
    std::atomic<long> lost{0}, twice{0};
    std::vector<std::thread> ts;
    for (int c = 0; c < callers; c++)
        ts.emplace_back([&, c] {
            for (int k = 0; k < calls; k++) {
                std::vector<std::atomic<int>> ran(members);
                for (auto& r : ran) r = 0;
                const int rc = pool.run([&](int i) -> int {
                    ran[i]++;
                    return (c + k + i) % 97 == 0 ? 7 : 0;
                });
                int want_rc = 0;
                for (int i = 0; i < members && !want_rc; i++) want_rc = (c + k + i) % 97 == 0 ? 7 : 0;
                for (int i = 0; i < members; i++) {
                    if (ran[i] == 0) lost++;
                    if (ran[i] > 1) twice++;
                }
                if (rc != want_rc) lost++;
            }
        });
    for (auto& t : ts) t.join();
    std::printf("%ld %ld\n", lost.load(), twice.load());
    return lost.load() || twice.load() ? 1 : 0;
}
