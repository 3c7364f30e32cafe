// fg_md5_host.hpp -- MD5 (RFC 1321) on a host core: the hash the reference's
// Md5 wrapper computes (std.crypto.hash.Md5 / OpenSSL, src/lib/md5.zig:3-31)
// over the raw WAV data bytes (wav_reader.zig:66).  One stream is a strictly
// sequential chain; a host core runs it ~10x faster than one GPU lane, so the
// host-buffer paths hash here, on a thread beside the GPU encode.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace fg {

struct HostMd5 {
    uint32_t h[4];
    uint64_t bytes;
    uint8_t buf[64];
    uint32_t fill;
    HostMd5() { reset(); }
    void reset();
    void update(const void *data, size_t len);
    void final(uint8_t digest[16]);  // pads, writes the digest, resets
};

// h->update(data, len) on the process-wide hashing pool (fg_md5_host.cpp): the bulk of a long
// update runs on a pool worker that hashes several callers' messages at once -- up to four chains
// interleaved step by step, or sixteen in the lanes of AVX-512 registers where the host has it
// (one MD5 chain leaves most of a core's issue width idle) -- so files encoded concurrently hash
// several times faster per core than one scalar chain each; more chains than fit the workers are
// time-sliced.  Blocks until done.
// FLACGPU_MD5_THREADS sets the worker count (default: the process's CPU share -- the cgroup quota,
// else the affinity mask's CPUs, divided by LOCAL_WORLD_SIZE when a launcher sets it and the
// process sees the whole machine; -1: no
// pool, each caller hashes its own chain).
void md5_pool_update(HostMd5 *h, const void *data, size_t len);

// hs[i]->update(data[i], lens[i]) for n independent chains on the pool, queued together (the
// plan path's host engine: every stream segment of a batch at once).  Blocks until all are done.
void md5_pool_update_many(HostMd5 *const *hs, const uint8_t *const *data, const size_t *lens, size_t n);

// the pool's default size: the cgroup quota (quota_cpus > 0) or the affinity mask's CPUs, divided
// by LOCAL_WORLD_SIZE only when the process sees every online CPU under no quota
int md5_pool_share_of(int quota_cpus, int aff, int online, const char *local_world);

// the pool's worker count (0: every caller hashes its own chain)
int md5_pool_workers();

// measured host MD5 rates: bytes/s per pool worker with pts[i] chains each (pts: 1, 2, 3, 4; with
// the AVX-512 path 1, 4, 8, 16); no pool: one chain's rate on the caller in every entry
// true if other chains were on the pool during the measurement (the rates may be low)
bool md5_measure_rates(double rate[4], uint32_t pts[4]);

// the AVX-512 sixteen-chain MD5 is in use (host support, FLACGPU_MD5_AVX512 != 0)
bool md5_avx512();

}  // namespace fg
