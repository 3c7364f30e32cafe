// sharded_encode_test.cpp -- the multi-rank encode through the C ABI only, the way a
// non-Python host (the reference's Zig CLI, wav2flac.zig:10-97) would drive BASELINE config 4:
// one process per GPU, every rank calls flacgpu_encode_frames_sharded with the whole stream,
// libflacgpu.so gathers the frames over its own RCCL communicator, and rank 0 writes the file
// (73-byte header with STREAMINFO replayed from the per-frame sizes in frame order,
// metadata.zig:35-40, and the stream MD5, encoder.zig:168-170).
//
// Usage: sharded_encode_test <pcm.raw> <channels> <bits> <rate> <world> <max_frames> <out.flac>
// The parent forks the other ranks BEFORE any HIP or RCCL call, then hands them the
// communicator id through a pipe.  Rank r runs on HIP device r.
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "flacgpu.h"

namespace {

int run_rank(int rank, int world, const uint8_t id[FLACGPU_COMM_ID_BYTES], const std::vector<uint8_t> &pcm,
             uint32_t ch, uint32_t bits, uint32_t rate, uint32_t max_frames, const char *out_path) {
    const uint32_t B = bits / 8;
    const uint64_t n = pcm.size() / (ch * B);
    flacgpu_config cfg = flacgpu_config_default(ch, bits, rate);
    flacgpu_ctx *ctx = nullptr;
    int rc = flacgpu_open(rank, &cfg, max_frames, &ctx);
    if (rc) {
        std::fprintf(stderr, "rank %d: open: %s\n", rank, flacgpu_strerror(rc));
        return 1;
    }
    flacgpu_comm *comm = nullptr;
    if ((rc = flacgpu_comm_init(id, world, rank, rank, &comm))) {
        std::fprintf(stderr, "rank %d: comm_init: %s\n", rank, flacgpu_strerror(rc));
        flacgpu_close(ctx);
        return 1;
    }
    const uint64_t nf = (n + 4095) / 4096;
    std::vector<uint8_t> frames(rank == 0 ? nf * flacgpu_frame_bound_bytes(&cfg) + 64 : 0);
    std::vector<uint32_t> sizes(rank == 0 ? nf + 1 : 0);
    size_t len = 0;
    rc = flacgpu_encode_frames_sharded(ctx, comm, pcm.data(), B, n, 0, frames.data(), frames.size(), &len,
                                       sizes.data());
    int status = 0;
    if (rc) {
        std::fprintf(stderr, "rank %d: encode_frames_sharded: %s\n", rank, flacgpu_strerror(rc));
        status = 1;
    } else if (rank == 0) {
        flacgpu_streaminfo si;
        flacgpu_streaminfo_init(&si, rate, ch, bits, n, 4096);
        for (uint64_t f = 0; f < nf; f++) flacgpu_streaminfo_update_frame_size(&si, sizes[f]);
        flacgpu_md5_init(ctx);
        flacgpu_md5_update(ctx, pcm.data(), pcm.size());
        flacgpu_md5_final(ctx, si.md5);
        uint8_t head[42], vorbis[31];
        const size_t hl = flacgpu_header_bytes(&si, 0, head), vl = flacgpu_vorbis_comment_bytes(1, vorbis);
        std::FILE *o = std::fopen(out_path, "wb");
        if (!o) {
            status = 1;
        } else {
            std::fwrite(head, 1, hl, o);
            std::fwrite(vorbis, 1, vl, o);
            std::fwrite(frames.data(), 1, len, o);
            std::fclose(o);
        }
    } else if (len != 0) {
        std::fprintf(stderr, "rank %d: out_len %zu on a non-root rank\n", rank, len);
        status = 1;
    }
    flacgpu_comm_destroy(comm);
    flacgpu_close(ctx);
    return status;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc != 8) {
        std::fprintf(stderr, "usage: %s pcm channels bits rate world max_frames out\n", argv[0]);
        return 2;
    }
    const uint32_t ch = std::atoi(argv[2]), bits = std::atoi(argv[3]), rate = std::atoi(argv[4]);
    const int world = std::atoi(argv[5]);
    const uint32_t max_frames = std::atoi(argv[6]);
    std::FILE *f = std::fopen(argv[1], "rb");
    if (!f || world < 1) return 2;
    std::vector<uint8_t> pcm;
    uint8_t tmp[1 << 16];
    size_t r;
    while ((r = std::fread(tmp, 1, sizeof tmp, f)) > 0) pcm.insert(pcm.end(), tmp, tmp + r);
    std::fclose(f);
    // fork the other ranks first: no HIP / RCCL state exists yet in any process
    std::vector<int> pipes(2 * world, -1);
    std::vector<pid_t> kids;
    int rank = 0;
    for (int k = 1; k < world; k++) {
        if (pipe(&pipes[2 * k]) != 0) return 2;
        const pid_t p = fork();
        if (p < 0) return 2;
        if (p == 0) {
            rank = k;
            break;
        }
        close(pipes[2 * k]);
        kids.push_back(p);
    }
    uint8_t id[FLACGPU_COMM_ID_BYTES];
    if (rank == 0) {
        const int rc = flacgpu_comm_unique_id(id);
        if (rc) std::fprintf(stderr, "comm_unique_id: %s\n", flacgpu_strerror(rc));
        for (int k = 1; k < world; k++) {
            // a failed id is still sent (zeros): the children fail their init instead of waiting
            if (write(pipes[2 * k + 1], id, sizeof id) != (ssize_t)sizeof id) return 2;
            close(pipes[2 * k + 1]);
        }
        if (rc) {
            for (pid_t p : kids) waitpid(p, nullptr, 0);
            return 1;
        }
    } else {
        close(pipes[2 * rank + 1]);
        size_t got = 0;
        while (got < sizeof id) {
            const ssize_t k = read(pipes[2 * rank], id + got, sizeof id - got);
            if (k <= 0) _exit(2);
            got += (size_t)k;
        }
        _exit(run_rank(rank, world, id, pcm, ch, bits, rate, max_frames, argv[7]));
    }
    int status = run_rank(0, world, id, pcm, ch, bits, rate, max_frames, argv[7]);
    for (pid_t p : kids) {
        int st = 0;
        waitpid(p, &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) status = 1;
    }
    return status;
}
