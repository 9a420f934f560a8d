// fpldpc_sim_plan.hpp -- frame partition and ordered stop rule of the BER/FER simulation over one
// or several decoders (fpldpc_ber_sim, fpldpc_ber_sim_multi).  Header-only, no HIP: the CPU test
// tests/cpp/sim_plan_test.cpp checks it against the reference's serial frame loop.
//
// The reference decodes frame after frame and stops at the frame whose decode brings the frame
// error count to the limit (PerfTest.cpp:97-135).  Here frames go out in rounds: in round r, rank
// i decodes frames [first + (r*ndev + i)*chunk, +chunk) (clipped to the frame limit), so every frame
// keeps its place in the one channel stream (frame f uses draws [f*n, (f+1)*n)) whatever the rank
// count.  After a round the ranks' chunk sums, taken in rank order, say whether the stop frame lies
// in this round and on which rank; that rank alone scans its chunk for the exact frame.  Counters
// over frames [first, stop] then equal the serial loop's for any rank count and chunk size.
#pragma once
#include <cstdint>

namespace fpldpc {
namespace plan {

struct Range {
    int64_t first = 0;
    int64_t frames = 0;
};

// Frames of rank `rank` in round `round` (frames == 0: nothing for this rank).
inline Range rank_range(int64_t first, int64_t frame_end, int chunk, int ndev, int64_t round, int rank) {
    Range r;
    r.first = first + (round * ndev + rank) * (int64_t)chunk;
    const int64_t left = frame_end - r.first;
    r.frames = left <= 0 ? 0 : (left < chunk ? left : chunk);
    return r;
}

// Does round `round` hold any frame at all (its rank 0 range is not empty)?
inline bool round_has_frames(int64_t first, int64_t frame_end, int chunk, int ndev, int64_t round) {
    return rank_range(first, frame_end, chunk, ndev, round, 0).frames > 0;
}

// Counters of the serial loop (PerfTest.cpp:125-133): blkerror > 0 makes a frame error.
struct Sums {
    int64_t bit_errors = 0, frame_errors = 0, frames = 0, iter_sum = 0;
    void add_frame(int64_t blk, int64_t it) {
        ++frames;
        iter_sum += it;
        bit_errors += blk;
        frame_errors += blk > 0;
    }
    void add(const Sums &o) {
        bit_errors += o.bit_errors;
        frame_errors += o.frame_errors;
        frames += o.frames;
        iter_sum += o.iter_sum;
    }
};

// Sums over a chunk's frames in order, stopping after the frame that brings prior_fe plus the
// chunk's frame errors to `need` (need <= 0: no limit).  Returns that frame's index, or -1 when
// the limit is not reached inside the chunk (then *s covers the whole chunk).
inline int64_t scan_chunk(const int32_t *blk, const int32_t *its, int64_t frames, int64_t prior_fe, int64_t need,
                          Sums *s) {
    Sums t;
    for (int64_t f = 0; f < frames; ++f) {
        t.add_frame(blk[f], its[f]);
        if (need > 0 && prior_fe + t.frame_errors >= need) {
            *s = t;
            return f;
        }
    }
    *s = t;
    return -1;
}

// The rank (in rank order) whose chunk holds the stop frame of this round, or -1: `all` are the
// ranks' whole-chunk sums, prior_fe the frame errors counted before the round.
inline int stop_rank(const Sums *all, int ndev, int64_t prior_fe, int64_t need) {
    if (need <= 0) return -1;
    int64_t fe = prior_fe;
    for (int i = 0; i < ndev; ++i) {
        fe += all[i].frame_errors;
        if (fe >= need) return i;
    }
    return -1;
}

// The counter exchange (include/fpldpc.h FPLDPC_COLL_*): RCCL is tried when asked for, or under
// AUTO for several decoders on distinct devices.
constexpr int kCollAuto = 0, kCollRccl = 1, kCollHost = 2;
inline bool try_rccl(int requested, bool distinct_devices, int ndev) {
    return requested == kCollRccl || (requested == kCollAuto && distinct_devices && ndev > 1);
}
// The exchange that runs after the communicator set-up (reported as collective_used), or -1: the
// call fails (RCCL asked for explicitly and not available).  AUTO falls back to host memory.
inline int exchange_after_init(int requested, bool tried_rccl, bool init_ok) {
    if (!tried_rccl) return kCollHost;
    if (init_ok) return kCollRccl;
    return requested == kCollAuto ? kCollHost : -1;
}

}  // namespace plan
}  // namespace fpldpc
