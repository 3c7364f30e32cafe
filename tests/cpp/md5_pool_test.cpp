// The host hashing pool (fg_md5_host.cpp md5_pool_update) against one plain HostMd5 chain per
// message: many caller threads at once, ragged lengths, updates split at odd offsets (partial
// blocks carried), worker counts from FLACGPU_MD5_THREADS, and a forked child (the pool's workers
// do not exist there: the child must hash on its own thread, not wait forever for them).
// Prints "ok" or the first mismatch.
#include <stdio.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <random>
#include <thread>
#include <vector>

#include "../../zig-flac_amd/csrc/fg_md5_host.hpp"

int main() {
    const int n_msgs = 24;
    std::mt19937_64 rng(12345);
    std::vector<std::vector<uint8_t>> msgs(n_msgs);
    for (int i = 0; i < n_msgs; i++) {
        const size_t len = (i % 5 == 0) ? (size_t)(rng() % 300) : (size_t)(rng() % (3u << 20)) + 4096u * (i % 3);
        msgs[i].resize(len);
        for (auto &b : msgs[i]) b = (uint8_t)rng();
    }
    std::vector<std::array<uint8_t, 16>> want(n_msgs), got(n_msgs);
    for (int i = 0; i < n_msgs; i++) {
        fg::HostMd5 h;
        h.update(msgs[i].data(), msgs[i].size());
        h.final(want[i].data());
    }
    for (int round = 0; round < 3; round++) {
        std::vector<std::thread> th;
        for (int i = 0; i < n_msgs; i++)
            th.emplace_back([&, i, round] {
                fg::HostMd5 h;
                const size_t n = msgs[i].size();
                // split into up to three updates at odd offsets (partial blocks carried over)
                const size_t a = round == 0 ? n : (n * (round + 1)) / 7, b = round == 2 ? a + (n - a) / 3 + 1 : n;
                fg::md5_pool_update(&h, msgs[i].data(), a);
                if (b <= n) fg::md5_pool_update(&h, msgs[i].data() + a, b - a);
                if (b < n) fg::md5_pool_update(&h, msgs[i].data() + b, n - b);
                h.final(got[i].data());
            });
        for (auto &t : th) t.join();
        for (int i = 0; i < n_msgs; i++)
            if (memcmp(got[i].data(), want[i].data(), 16) != 0) {
                printf("mismatch: round %d message %d (%zu bytes)\n", round, i, msgs[i].size());
                return 1;
            }
    }
    // fork after the pool's workers started: the child hashes inline (no worker threads exist in
    // it); a child that queued its job would block forever, so the parent bounds the wait
    const pid_t pid = fork();
    if (pid == 0) {
        alarm(20);
        fg::HostMd5 h;
        fg::md5_pool_update(&h, msgs[1].data(), msgs[1].size());
        std::array<uint8_t, 16> d;
        h.final(d.data());
        _exit(memcmp(d.data(), want[1].data(), 16) == 0 ? 0 : 3);
    }
    int st = 0;
    if (pid < 0 || waitpid(pid, &st, 0) != pid || !WIFEXITED(st) || WEXITSTATUS(st) != 0) {
        printf("forked child failed (status %d)\n", st);
        return 1;
    }
    printf("ok\n");
    return 0;
}
