// sim_plan_test.cpp -- CPU check of the multi-device simulation's partition and ordered stop rule
// (fixedpointldpc_amd/csrc/fpldpc_sim_plan.hpp) against the reference's serial frame loop
// (PerfTest.cpp:97-135: decode frame after frame, count blkerror > 0 as a frame error, stop at the
// frame that reaches the limit).  Random per-frame outcomes; ranks emulated round by round exactly
// as rank_loop (fpldpc_sim.cpp) runs them.  Exit 0 = all trials agree.
#include <cstdio>
#include <random>
#include <vector>

#include "fpldpc_sim_plan.hpp"

using namespace fpldpc::plan;

int main() {
    std::mt19937_64 rng(20261016);
    int bad = 0, trials = 0;
    for (int t = 0; t < 20000; ++t) {
        const int total = 1 + (int)(rng() % 3000);
        std::vector<int32_t> blk(total), its(total);
        const int per_mille = (int)(rng() % 400);
        for (int f = 0; f < total; ++f) {
            const bool err = (int)(rng() % 1000) < per_mille;
            blk[f] = err ? 1 + (int)(rng() % 20) : 0;
            its[f] = (int)(rng() % 31);
        }
        const int64_t first = (int64_t)(rng() % 50);
        const int ndev = 1 + (int)(rng() % 8), chunk = 1 + (int)(rng() % 64);
        int64_t need = (int64_t)(rng() % 60), max_frames = (int64_t)(rng() % (total + 1));
        if (need == 0 && max_frames == 0) max_frames = 1;
        // frames beyond the generated outcomes are never needed: clamp the limit to them
        const int64_t avail = total - first;
        if (avail <= 0) continue;
        if (max_frames == 0 || max_frames > avail) max_frames = avail;
        const int64_t frame_end = first + max_frames;
        ++trials;
        // serial loop
        Sums ser;
        for (int64_t f = first; f < frame_end; ++f) {
            ser.add_frame(blk[f], its[f]);
            if (need > 0 && ser.frame_errors >= need) break;
        }
        // rounds
        Sums tot;
        for (int64_t round = 0;; ++round) {
            std::vector<Sums> sums(ndev);
            std::vector<Range> rg(ndev);
            for (int i = 0; i < ndev; ++i) {
                rg[i] = rank_range(first, frame_end, chunk, ndev, round, i);
                for (int64_t f = 0; f < rg[i].frames; ++f) sums[i].add_frame(blk[rg[i].first + f], its[rg[i].first + f]);
            }
            const int sr = stop_rank(sums.data(), ndev, tot.frame_errors, need);
            if (sr < 0) {
                for (auto &s : sums) tot.add(s);
                if (!round_has_frames(first, frame_end, chunk, ndev, round + 1)) break;
                continue;
            }
            int64_t prior = tot.frame_errors;
            for (int i = 0; i < sr; ++i) {
                tot.add(sums[i]);
                prior += sums[i].frame_errors;
            }
            Sums part;
            const int64_t at = scan_chunk(&blk[rg[sr].first], &its[rg[sr].first], rg[sr].frames, prior, need, &part);
            if (at < 0) ++bad;  // the stop rank must find its frame
            tot.add(part);
            break;
        }
        if (tot.frames != ser.frames || tot.frame_errors != ser.frame_errors || tot.bit_errors != ser.bit_errors ||
            tot.iter_sum != ser.iter_sum) {
            if (bad < 5)
                fprintf(stderr, "mismatch: first %lld ndev %d chunk %d need %lld max %lld: %lld/%lld frames\n",
                        (long long)first, ndev, chunk, (long long)need, (long long)max_frames, (long long)tot.frames,
                        (long long)ser.frames);
            ++bad;
        }
    }
    // the counter exchange: RCCL when asked for, or AUTO over distinct devices; a failed set-up fails
    // an explicit RCCL request and falls back to (and reports) the host exchange under AUTO
    const bool ok_try = try_rccl(kCollRccl, false, 1) && try_rccl(kCollAuto, true, 2) && !try_rccl(kCollAuto, true, 1) &&
                        !try_rccl(kCollAuto, false, 3) && !try_rccl(kCollHost, true, 8);
    const bool ok_after = exchange_after_init(kCollRccl, true, true) == kCollRccl &&
                          exchange_after_init(kCollRccl, true, false) == -1 &&
                          exchange_after_init(kCollAuto, true, false) == kCollHost &&
                          exchange_after_init(kCollAuto, true, true) == kCollRccl &&
                          exchange_after_init(kCollAuto, false, true) == kCollHost &&
                          exchange_after_init(kCollHost, false, true) == kCollHost;
    if (!ok_try || !ok_after) {
        fprintf(stderr, "collective choice: try %d after-init %d\n", ok_try, ok_after);
        ++bad;
    }
    printf("%d trials, %d mismatches\n", trials, bad);
    return bad != 0;
}
