// fpldpc_sim.cpp -- ordered BER/FER simulation around one or several GPU decoders
// (fpldpc_ber_sim, fpldpc_ber_sim_multi).
//
// The reference harness decodes one frame at a time and stops at the frame whose decode brings the
// frame-error count to 100 (PerfTest.cpp:97-135, 275-311, 385-426, 485-511, 574-600).  Here frames
// are decoded in chunks: each rank (one decoder, one device, one host thread) holds two pinned /
// device buffer pairs on its decoder's stream, so that the host generates the next chunk's LLRs
// while the GPU decodes this one (or, with device_channel, the LLRs are generated on the device in
// the same stream, fpldpc_gen.hip).  Rounds, ranges and the stop rule are fpldpc_sim_plan.hpp's:
// per round the ranks exchange their chunk sums (an all-gather), the rank holding the stop frame
// scans its chunk for it, and one all-reduce adds the contributions -- so every counter equals the
// serial loop's for any number of ranks.  With decoders on distinct devices the exchange is RCCL
// (ncclCommInitAll in this process, collectives on each decoder's stream, over xGMI on an MI355X
// node); decoders sharing a device exchange through host memory.  Frames of the last round past the
// stop frame are decoded but not counted.
//
// Two chunks in flight per rank: the two slots decode on two decoders (the caller's and a twin with
// the same code and parameters) on their own streams, and round r+1's chunk is submitted before
// round r's is waited for, so the next chunk's workgroups take the CUs that a chunk's last frames
// leave idle (with early termination a chunk ends on a few frames running max_iter iterations
// alone).  The exchange runs on a third stream.  Counters are unchanged: chunks are still counted
// in round order, and a chunk decoded past the stop frame is drained, not counted.
// FPLDPC_SIM_OVERLAP=0 submits each chunk after the previous round's exchange, on one decoder.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fpldpc_internal.hpp"
#include "fpldpc_sim_plan.hpp"
#include "fpldpc_testing.h"

using namespace fpldpc;

namespace {

#define SIM_TRY(expr)                                          \
    do {                                                       \
        hipError_t _e = (expr);                                \
        if (_e != hipSuccess) return fail_hip((int)_e, #expr); \
    } while (0)

struct Slot {
    int16_t *h_llr = nullptr;
    int32_t *h_out = nullptr;  // [chunk] bit errors, [chunk] iterations, [1] int16 overflow count
    int16_t *d_llr = nullptr;
    int32_t *d_out = nullptr;
    hipEvent_t done = nullptr;
    int64_t frames = 0;
    int64_t first = 0;
    fpldpc_decoder_t dec = nullptr;  // decodes this slot's chunks, on its own stream
};

// One rank: a decoder, its stream, two chunk slots.
struct Rank {
    fpldpc_decoder_t dec = nullptr;
    fpldpc_decoder_t twin = nullptr;  // second decoder (two chunks in flight), owned here
    hipStream_t xs = nullptr;         // the exchange's stream when two chunks are in flight
    bool overlap = false;
    const fpldpc_sim_params *sp = nullptr;
    int chunk = 0, n = 0;
    Slot s[2];
    int32_t *d_forced = nullptr;
    const uint8_t *d_cw = nullptr;
    int64_t decoded = 0;
    ~Rank() {
        // a rank that left early (an error) may still have a chunk in flight: let it finish before
        // its buffers and the twin decoder go
        for (auto &x : s)
            if (x.dec) (void)hipStreamSynchronize(x.dec->stream);
        if (twin) (void)fpldpc_decoder_destroy(twin);
        if (xs) (void)hipStreamDestroy(xs);
        (void)hipFree(d_forced);
        for (auto &x : s) {
            (void)hipHostFree(x.h_llr);
            (void)hipHostFree(x.h_out);
            (void)hipFree(x.d_llr);
            (void)hipFree(x.d_out);
            if (x.done) (void)hipEventDestroy(x.done);
        }
    }
    hipStream_t exchange_stream() const { return xs ? xs : dec->stream; }
    int setup() {  // on the decoder's device
        const size_t llr_bytes = (size_t)chunk * n * sizeof(int16_t);
        s[0].dec = s[1].dec = dec;
        if (overlap) {
            int st = decoder_create_twin(dec, &twin);
            if (st) return st;
            s[1].dec = twin;
            SIM_TRY(hipStreamCreateWithFlags(&xs, hipStreamNonBlocking));
        }
        for (auto &x : s) {
            if (!sp->device_channel) SIM_TRY(hipHostMalloc((void **)&x.h_llr, llr_bytes, hipHostMallocDefault));
            SIM_TRY(hipHostMalloc((void **)&x.h_out, ((size_t)chunk * 2 + 1) * sizeof(int32_t), hipHostMallocDefault));
            SIM_TRY(hipMalloc((void **)&x.d_llr, llr_bytes));
            SIM_TRY(hipMalloc((void **)&x.d_out, ((size_t)chunk * 2 + 1) * sizeof(int32_t)));
            SIM_TRY(hipEventCreateWithFlags(&x.done, hipEventDisableTiming));
        }
        if (sp->device_channel) {
            if (sp->codeword) {
                SIM_TRY(hipMalloc((void **)&d_forced, sizeof(int32_t) * std::max(sp->n_forced, 0) + n));
                d_cw = reinterpret_cast<const uint8_t *>(d_forced + std::max(sp->n_forced, 0));
                SIM_TRY(hipMemcpy((void *)d_cw, sp->codeword, n, hipMemcpyHostToDevice));
            } else if (sp->n_forced > 0) {
                SIM_TRY(hipMalloc((void **)&d_forced, sizeof(int32_t) * sp->n_forced));
            }
            if (sp->n_forced > 0)
                SIM_TRY(hipMemcpy(d_forced, sp->forced_index, sizeof(int32_t) * sp->n_forced, hipMemcpyHostToDevice));
        }
        if (sp->count_mode == FPLDPC_COUNT_BITS) {
            int st = fpldpc_set_reference(dec, sp->info_index, sp->info_bits, sp->k);
            if (!st && twin) st = fpldpc_set_reference(twin, sp->info_index, sp->info_bits, sp->k);
            return st;
        }
        return FPLDPC_OK;
    }
    // Host channel: the chunk's LLRs on host threads (device channel: in submit).
    int generate(Slot &x, plan::Range r) {
        x.first = r.first;
        x.frames = r.frames;
        if (x.frames <= 0 || sp->device_channel) return FPLDPC_OK;
        int st = fpldpc_channel_llr_host(sp->seed, x.first, (int32_t)x.frames, n, sp->snr, sp->sigma, sp->frac_bits,
                                         sp->codeword, x.h_llr, FPLDPC_LLR_I16, sp->host_threads);
        if (st) return st;
        for (int64_t f = 0; f < x.frames; f++)
            for (int i = 0; i < sp->n_forced; i++) x.h_llr[(size_t)f * n + sp->forced_index[i]] = (int16_t)sp->forced_llr;
        return FPLDPC_OK;
    }
    int submit(Slot &x) {
        if (x.frames <= 0) return FPLDPC_OK;
        hipStream_t st = x.dec->stream;
        int r;
        if (sp->device_channel) {
            int32_t *ovf = x.d_out + 2 * (size_t)chunk;
            SIM_TRY(hipMemsetAsync(ovf, 0, sizeof(int32_t), st));
            if ((r = launch_channel(sp->seed, x.first, (int)x.frames, n, sp->snr, sp->sigma, sp->frac_bits, d_cw, 0,
                                    x.d_llr, FPLDPC_LLR_I16, ovf, st)))
                return r;
            if (sp->n_forced > 0 &&
                (r = launch_force_llr(x.d_llr, (int)x.frames, n, d_forced, sp->n_forced, (int16_t)sp->forced_llr, st)))
                return r;
            SIM_TRY(hipMemcpyAsync(x.h_out + 2 * (size_t)chunk, ovf, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        } else {
            SIM_TRY(hipMemcpyAsync(x.d_llr, x.h_llr, (size_t)x.frames * n * sizeof(int16_t), hipMemcpyHostToDevice, st));
        }
        r = fpldpc_decode(x.dec, x.d_llr, FPLDPC_LLR_I16, (int32_t)x.frames, nullptr, x.d_out + chunk, nullptr, nullptr,
                          sp->count_mode == FPLDPC_COUNT_BITS ? x.d_out : nullptr, nullptr, st);
        if (r) return r;
        if (sp->count_mode == FPLDPC_COUNT_BITS)
            SIM_TRY(hipMemcpyAsync(x.h_out, x.d_out, (size_t)x.frames * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        SIM_TRY(hipMemcpyAsync(x.h_out + chunk, x.d_out + chunk, (size_t)x.frames * sizeof(int32_t),
                               hipMemcpyDeviceToHost, st));
        SIM_TRY(hipEventRecord(x.done, st));
        return FPLDPC_OK;
    }
    int wait(Slot &x) {
        if (x.frames <= 0) return FPLDPC_OK;
        SIM_TRY(hipEventSynchronize(x.done));
        if (sp->device_channel && x.h_out[2 * (size_t)chunk] != 0)
            return fail(FPLDPC_ERR_ARG, "LLR does not fit int16");  // as the host channel
        decoded += x.frames;
        return FPLDPC_OK;
    }
    // blkerror per frame: calculateBER or decode_fixpoint's return value
    const int32_t *blk(const Slot &x) const { return sp->count_mode == FPLDPC_COUNT_BITS ? x.h_out : x.h_out + chunk; }
    const int32_t *its(const Slot &x) const { return x.h_out + chunk; }
};

// Host barrier for the rank threads (generation count, reusable).  abort() releases every waiter
// for good: wait() then returns false, so a failed rank cannot leave the others blocked.
class Barrier {
  public:
    explicit Barrier(int n) : n_(n) {}
    bool wait() {
        std::unique_lock<std::mutex> l(m_);
        if (aborted_) return false;
        const uint64_t g = gen_;
        if (++count_ == n_) {
            count_ = 0;
            ++gen_;
            cv_.notify_all();
        } else {
            cv_.wait(l, [&] { return gen_ != g || aborted_; });
            return gen_ != g;  // completed, even if a rank that left it first has aborted since
        }
        return true;
    }
    void abort() {
        std::lock_guard<std::mutex> l(m_);
        aborted_ = true;
        cv_.notify_all();
    }

  private:
    std::mutex m_;
    std::condition_variable cv_;
    int n_, count_ = 0;
    uint64_t gen_ = 0;
    bool aborted_ = false;
};

constexpr int kWords = 5;  // exchanged per rank: 4 counters + a status / frames-decoded word

// The exchange between ranks.  Every rank makes the same sequence of calls.  A rank that fails
// anywhere calls abort(): host-mode waiters leave the barrier, and RCCL-mode ranks, which wait for
// their collectives by polling their own stream, abort their own communicator (from their own
// thread, so no communicator is freed under another thread) and return an error.
struct Exchange {
    int ndev = 1;
    Barrier bar{1};
    std::atomic<bool> aborted{false};
    // host mode: double-buffered slots, indexed by call parity (a barrier separates the calls)
    std::vector<int64_t> slots;
    std::vector<int> calls;
    // RCCL mode
    std::vector<ncclComm_t> comms;
    std::vector<int64_t *> dbuf;  // per rank: [kWords] send + [ndev * kWords] receive
    bool rccl = false;
    Exchange(int n, bool use_rccl) : ndev(n), bar(n), slots(2 * (size_t)n * kWords), calls(n, 0), rccl(use_rccl) {}
    ~Exchange() { release(); }
    void release() {
        for (auto *p : dbuf) (void)hipFree(p);
        dbuf.clear();
        for (auto c : comms)  // after a failure, peers may never join a collective: abort, don't destroy
            if (c) (void)(aborted ? ncclCommAbort(c) : ncclCommDestroy(c));
        comms.clear();
    }
    void abort() {
        aborted = true;
        bar.abort();
    }
    int init(const std::vector<fpldpc_decoder_t> &decs, bool injected_failure) {
        if (!rccl) return FPLDPC_OK;
        if (injected_failure) return fail(FPLDPC_ERR_HIP, "ncclCommInitAll: injected failure (fpldpc_testing_sim_inject)");
        std::vector<int> devs(ndev);
        for (int i = 0; i < ndev; ++i) devs[i] = decs[i]->device;
        comms.assign(ndev, nullptr);
        ncclResult_t r = ncclCommInitAll(comms.data(), ndev, devs.data());
        if (r != ncclSuccess) {
            comms.clear();
            return fail(FPLDPC_ERR_HIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
        }
        dbuf.assign(ndev, nullptr);
        for (int i = 0; i < ndev; ++i) {
            if (hipSetDevice(devs[i]) != hipSuccess) return fail(FPLDPC_ERR_HIP, "hipSetDevice");
            SIM_TRY(hipMalloc((void **)&dbuf[i], sizeof(int64_t) * kWords * (ndev + 1)));
        }
        return FPLDPC_OK;
    }
    // Wait for this rank's collective (RCCL mode) while watching for another rank's failure.
    int sync(int rank, hipStream_t st) {
        for (;;) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipSuccess) return FPLDPC_OK;
            if (q != hipErrorNotReady) return fail_hip((int)q, "hipStreamQuery (collective)");
            if (aborted) {
                (void)ncclCommAbort(comms[rank]);
                comms[rank] = nullptr;
                return fail(FPLDPC_ERR_HIP, "another rank of the simulation failed (collective aborted)");
            }
            std::this_thread::yield();
        }
    }
    // all[ndev][kWords] = every rank's `mine`, in rank order
    int allgather(int rank, hipStream_t st, const int64_t *mine, int64_t *all) {
        if (aborted) return fail(FPLDPC_ERR_HIP, "another rank of the simulation failed");
        if (rccl) {
            int64_t *send = dbuf[rank], *recv = dbuf[rank] + kWords;
            SIM_TRY(hipMemcpyAsync(send, mine, sizeof(int64_t) * kWords, hipMemcpyHostToDevice, st));
            ncclResult_t r = ncclAllGather(send, recv, kWords, ncclInt64, comms[rank], st);
            if (r != ncclSuccess) return fail(FPLDPC_ERR_HIP, std::string("ncclAllGather: ") + ncclGetErrorString(r));
            SIM_TRY(hipMemcpyAsync(all, recv, sizeof(int64_t) * kWords * ndev, hipMemcpyDeviceToHost, st));
            return sync(rank, st);
        }
        int64_t *buf = &slots[(size_t)(calls[rank]++ & 1) * ndev * kWords];
        memcpy(buf + (size_t)rank * kWords, mine, sizeof(int64_t) * kWords);
        if (!bar.wait()) return fail(FPLDPC_ERR_HIP, "another rank of the simulation failed");
        memcpy(all, buf, sizeof(int64_t) * kWords * ndev);
        return FPLDPC_OK;
    }
    // sum over ranks of `mine` (kWords)
    int allreduce(int rank, hipStream_t st, const int64_t *mine, int64_t *sum) {
        if (aborted) return fail(FPLDPC_ERR_HIP, "another rank of the simulation failed");
        if (rccl) {
            int64_t *buf = dbuf[rank];
            SIM_TRY(hipMemcpyAsync(buf, mine, sizeof(int64_t) * kWords, hipMemcpyHostToDevice, st));
            ncclResult_t r = ncclAllReduce(buf, buf, kWords, ncclInt64, ncclSum, comms[rank], st);
            if (r != ncclSuccess) return fail(FPLDPC_ERR_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
            SIM_TRY(hipMemcpyAsync(sum, buf, sizeof(int64_t) * kWords, hipMemcpyDeviceToHost, st));
            return sync(rank, st);
        }
        std::vector<int64_t> all((size_t)ndev * kWords);
        const int e = allgather(rank, st, mine, all.data());
        if (e) return e;
        for (int w = 0; w < kWords; ++w) {
            sum[w] = 0;
            for (int i = 0; i < ndev; ++i) sum[w] += all[(size_t)i * kWords + w];
        }
        return FPLDPC_OK;
    }
};

struct Shared {
    const fpldpc_sim_params *sp = nullptr;
    int ndev = 1, chunk = 0;
    int64_t frame_end = 0;
    Exchange *ex = nullptr;
    std::vector<Rank *> ranks;  // on_frame: rank 0's thread reads every rank's slot in frame order
    // per rank outcome
    std::vector<int> status;
    std::vector<std::string> message;
    plan::Sums result;
    int64_t decoded = 0;
    int fail_rank = -1;  // fpldpc_testing_sim_inject (include/fpldpc_testing.h)
    int64_t fail_round = 0;
    bool fail_abrupt = false;
};

// Test-only fault injection (include/fpldpc_testing.h), set by an explicit call, never from the
// environment.
struct Inject {
    std::atomic<int> fail_rank{-1};
    std::atomic<int64_t> fail_round{0};
    std::atomic<bool> abrupt{false};
    std::atomic<int> comm_init{0};  // 1: ncclCommInitAll fails; 2: also AUTO attempts RCCL on one device
};
Inject g_inject;

void pack(const plan::Sums &s, int64_t w4, int64_t *out) {
    out[0] = s.bit_errors;
    out[1] = s.frame_errors;
    out[2] = s.frames;
    out[3] = s.iter_sum;
    out[4] = w4;
}
plan::Sums unpack(const int64_t *w) {
    plan::Sums s;
    s.bit_errors = w[0];
    s.frame_errors = w[1];
    s.frames = w[2];
    s.iter_sum = w[3];
    return s;
}

// One rank's frame loop.  Every rank runs the same rounds and the same collective calls; a rank
// that fails reports its status through the round's all-gather so that all stop together.
int rank_loop(Shared &sh, int rank) {
    Rank &R = *sh.ranks[rank];
    const fpldpc_sim_params *sp = sh.sp;
    const int ndev = sh.ndev;
    hipStream_t st = R.exchange_stream();
    const int64_t need = sp->max_frame_errors;
    auto range = [&](int64_t round, int rk) {
        return plan::rank_range(sp->first_frame, sh.frame_end, sh.chunk, ndev, round, rk);
    };
    plan::Sums total;  // the counted frames before the current round (identical on every rank)
    int err = FPLDPC_OK;
    std::string own;  // this rank's first error message
    int cur = 0;
    int64_t round = 0;
    err = R.generate(R.s[0], range(0, rank));
    if (!err) err = R.submit(R.s[0]);
    std::vector<int64_t> all((size_t)ndev * kWords);
    int64_t mine[kWords], red[kWords];
    for (;;) {
        Slot &x = R.s[cur], &y = R.s[cur ^ 1];
        const bool more = plan::round_has_frames(sp->first_frame, sh.frame_end, sh.chunk, ndev, round + 1);
        y.frames = 0;
        if (!err && rank == sh.fail_rank && round == sh.fail_round) {
            err = fail(FPLDPC_ERR_HIP, "injected failure (fpldpc_testing_sim_inject)");
            own = fpldpc_last_error();
            if (sh.fail_abrupt) {
                for (const Slot &z : R.s) (void)hipStreamSynchronize(z.dec->stream);
                return err;
            }
        }
        // overlap: the next round's host channel while the GPU decodes this one, and with two
        // decoders the next round's decode as well
        if (!err && more) err = R.generate(y, range(round + 1, rank));
        if (!err && more && R.overlap) err = R.submit(y);
        if (!err) err = R.wait(x);
        if (err && own.empty()) own = fpldpc_last_error();
        plan::Sums loc;
        if (!err)
            for (int64_t f = 0; f < x.frames; ++f) loc.add_frame(R.blk(x)[f], R.its(x)[f]);
        pack(loc, err, mine);
        int e2 = sh.ex->allgather(rank, st, mine, all.data());
        if (e2 && err) return fail(err, own);  // this rank's own error, not the abort it caused
        if (e2) return e2;
        int first_err = FPLDPC_OK;
        for (int i = 0; i < ndev && !first_err; ++i) first_err = (int)all[(size_t)i * kWords + 4];
        if (first_err) return err ? err : fail(first_err, "another rank of the simulation failed");
        std::vector<plan::Sums> sums(ndev);
        for (int i = 0; i < ndev; ++i) sums[i] = unpack(&all[(size_t)i * kWords]);
        const int sr = plan::stop_rank(sums.data(), ndev, total.frame_errors, need);
        if (sp->on_frame) {  // frame order across ranks: rank 0's thread calls back for everyone
            if (!sh.ex->bar.wait()) return fail(FPLDPC_ERR_HIP, "another rank of the simulation failed");
            if (rank == 0) {
                plan::Sums run = total;
                for (int i = 0; i <= (sr < 0 ? ndev - 1 : sr); ++i) {
                    const Rank &Ri = *sh.ranks[i];
                    const Slot &xi = Ri.s[cur];
                    for (int64_t f = 0; f < xi.frames; ++f) {
                        sp->on_frame(sp->on_frame_ctx, xi.first + f, Ri.its(xi)[f], Ri.blk(xi)[f]);
                        run.add_frame(Ri.blk(xi)[f], Ri.its(xi)[f]);
                        if (i == sr && need > 0 && run.frame_errors >= need) break;
                    }
                }
            }
            if (!sh.ex->bar.wait()) return fail(FPLDPC_ERR_HIP, "another rank of the simulation failed");
        }
        if (sr < 0) {
            for (int i = 0; i < ndev; ++i) total.add(sums[i]);
            if (!more) {
                pack(plan::Sums(), R.decoded, mine);
                break;
            }
            if (!R.overlap) err = R.submit(y);
            cur ^= 1;
            ++round;
            continue;
        }
        // the stop frame lies in rank sr's chunk: ranks before it count whole chunks, rank sr up
        // to the stop frame, ranks after it nothing
        plan::Sums contrib;
        if (rank < sr) contrib = loc;
        if (rank == sr) {
            int64_t prior = total.frame_errors;
            for (int i = 0; i < sr; ++i) prior += sums[i].frame_errors;
            plan::scan_chunk(R.blk(x), R.its(x), x.frames, prior, need, &contrib);
        }
        pack(contrib, R.decoded, mine);
        break;
    }
    int e3 = sh.ex->allreduce(rank, st, mine, red);
    if (e3) return e3;
    total.add(unpack(red));
    // drain: a generated-but-not-submitted slot holds nothing on the device; a submitted one (two
    // chunks in flight, decoded past the stop frame) is waited for, not counted
    for (const Slot &z : R.s) SIM_TRY(hipStreamSynchronize(z.dec->stream));
    SIM_TRY(hipStreamSynchronize(st));
    if (rank == 0) {
        sh.result = total;
        sh.decoded = red[4];
    }
    return FPLDPC_OK;
}

int validate(fpldpc_decoder_t dec, const fpldpc_sim_params *sp) {
    const int n = dec->code.n;
    if (sp->max_frame_errors <= 0 && sp->max_frames <= 0)
        return fail(FPLDPC_ERR_ARG, "ber_sim needs max_frame_errors or max_frames");
    if (sp->count_mode != FPLDPC_COUNT_BITS && sp->count_mode != FPLDPC_COUNT_ITERS)
        return fail(FPLDPC_ERR_ARG, "bad count_mode");
    if (sp->count_mode == FPLDPC_COUNT_BITS && (sp->k <= 0 || !sp->info_index || !sp->info_bits))
        return fail(FPLDPC_ERR_ARG, "FPLDPC_COUNT_BITS needs info_index / info_bits");
    if (sp->n_forced < 0 || (sp->n_forced > 0 && !sp->forced_index)) return fail(FPLDPC_ERR_ARG, "bad forced list");
    for (int i = 0; i < sp->n_forced; i++)
        if (sp->forced_index[i] < 0 || sp->forced_index[i] >= n) return fail(FPLDPC_ERR_ARG, "forced index out of range");
    if (sp->forced_llr < -32768 || sp->forced_llr > 32767) return fail(FPLDPC_ERR_ARG, "forced_llr must fit int16");
    return FPLDPC_OK;
}

struct DeviceRestore {
    int d = -1;
    DeviceRestore() { (void)hipGetDevice(&d); }
    ~DeviceRestore() {
        if (d >= 0) (void)hipSetDevice(d);
    }
};

int run_sim(const fpldpc_decoder_t *decs, int ndev, const fpldpc_sim_params *sp, int collective, fpldpc_sim_result *out,
            int32_t *used) {
    if (!decs || ndev < 1 || !sp || !out) return fail(FPLDPC_ERR_ARG, "null argument");
    if (collective < FPLDPC_COLL_AUTO || collective > FPLDPC_COLL_HOST) return fail(FPLDPC_ERR_ARG, "bad collective");
    std::vector<fpldpc_decoder_t> dv(decs, decs + ndev);
    bool distinct = true;
    for (int i = 0; i < ndev; ++i) {
        if (!dv[i]) return fail(FPLDPC_ERR_ARG, "null decoder");
        if (dv[i]->code.n != dv[0]->code.n || dv[i]->code.m != dv[0]->code.m)
            return fail(FPLDPC_ERR_ARG, "decoders of different codes");
        for (int j = 0; j < i; ++j) {
            if (dv[j] == dv[i]) return fail(FPLDPC_ERR_ARG, "the same decoder twice (a decoder is single-stream)");
            distinct = distinct && dv[j]->device != dv[i]->device;
        }
        int st = validate(dv[i], sp);
        if (st) return st;
    }
    static_assert(FPLDPC_COLL_AUTO == plan::kCollAuto && FPLDPC_COLL_RCCL == plan::kCollRccl &&
                  FPLDPC_COLL_HOST == plan::kCollHost, "collective codes");
    // (test hook: comm_init == 2 makes AUTO attempt RCCL with a single decoder, so that its fallback
    // runs on a one-GPU box)
    const bool rccl = plan::try_rccl(collective, distinct, ndev) ||
                      (collective == FPLDPC_COLL_AUTO && ndev == 1 && g_inject.comm_init.load() == 2);
    if (rccl && !distinct) return fail(FPLDPC_ERR_ARG, "RCCL needs the decoders on distinct devices");
    const auto t0 = std::chrono::steady_clock::now();
    DeviceRestore restore;
    const char *ov = getenv("FPLDPC_SIM_OVERLAP");
    const bool overlap = !(ov && *ov == '0');

    Shared sh;
    sh.sp = sp;
    sh.ndev = ndev;
    sh.chunk = sp->chunk > 0 ? sp->chunk : 16384;
    if (sp->max_frames > 0) sh.chunk = (int)std::min<int64_t>(sh.chunk, sp->max_frames);
    sh.frame_end = sp->max_frames > 0 ? sp->first_frame + sp->max_frames : INT64_MAX;
    Exchange ex(ndev, rccl);
    sh.ex = &ex;
    std::vector<std::unique_ptr<Rank>> ranks(ndev);
    for (int i = 0; i < ndev; ++i) {
        ranks[i].reset(new Rank);
        ranks[i]->dec = dv[i];
        ranks[i]->sp = sp;
        ranks[i]->chunk = sh.chunk;
        ranks[i]->n = dv[i]->code.n;
        ranks[i]->overlap = overlap;
        if (hipSetDevice(dv[i]->device) != hipSuccess) return fail(FPLDPC_ERR_HIP, "hipSetDevice failed");
        int st = ranks[i]->setup();
        if (st) return st;
        sh.ranks.push_back(ranks[i].get());
    }
    int st = ex.init(dv, g_inject.comm_init.load() != 0);
    const int coll_used = plan::exchange_after_init(collective, rccl, st == FPLDPC_OK);
    if (coll_used < 0) return st;
    if (st) {  // AUTO: identical counters without RCCL, through host memory
        fprintf(stderr, "fpldpc_ber_sim_multi: %s; exchanging the counters through host memory instead\n",
                fpldpc_last_error());
        ex.release();
        ex.rccl = false;
        st = FPLDPC_OK;
    }
    sh.fail_rank = g_inject.fail_rank.load();
    sh.fail_round = g_inject.fail_round.load();
    sh.fail_abrupt = g_inject.abrupt.load();
    sh.status.assign(ndev, FPLDPC_OK);
    sh.message.assign(ndev, std::string());
    if (ndev == 1) {  // in the calling thread (its device and error state)
        if (hipSetDevice(dv[0]->device) != hipSuccess) return fail(FPLDPC_ERR_HIP, "hipSetDevice failed");
        st = rank_loop(sh, 0);
        if (st) return st;
    } else {
        std::vector<std::thread> th;
        for (int i = 0; i < ndev; ++i)
            th.emplace_back([&, i] {
                if (hipSetDevice(dv[i]->device) != hipSuccess) {
                    sh.status[i] = fail(FPLDPC_ERR_HIP, "hipSetDevice failed");
                } else {
                    sh.status[i] = rank_loop(sh, i);
                }
                if (sh.status[i]) {
                    sh.message[i] = fpldpc_last_error();
                    ex.abort();  // every failure ends the others' waits (barrier, polled collectives)
                }
            });
        for (auto &t : th) t.join();
        // report the rank that failed first-hand, not one that only saw the abort
        for (int pass = 0; pass < 2; ++pass)
            for (int i = 0; i < ndev; ++i)
                if (sh.status[i] && (pass == 1 || sh.message[i].find("another rank") == std::string::npos))
                    return fail(sh.status[i], "rank " + std::to_string(i) + ": " + sh.message[i]);
    }
    fpldpc_sim_result r{};
    r.bit_errors = sh.result.bit_errors;
    r.frame_errors = sh.result.frame_errors;
    r.frames = sh.result.frames;
    r.iter_sum = sh.result.iter_sum;
    r.frames_decoded = sh.decoded;
    r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    *out = r;
    if (used) *used = coll_used;  // what ran, after any AUTO fallback
    return FPLDPC_OK;
}

}  // namespace

extern "C" {

void fpldpc_sim_params_default(fpldpc_sim_params *p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->seed = 123456789;  // rngs.cpp:45
    p->frac_bits = 4;     // ArrayLDPCMacro.h:36
    p->max_frame_errors = 100;  // PerfTest.cpp:97
    p->count_mode = FPLDPC_COUNT_BITS;
}

int fpldpc_ber_sim(fpldpc_decoder_t dec, const fpldpc_sim_params *sp, fpldpc_sim_result *out) {
    if (!dec) return fail(FPLDPC_ERR_ARG, "null argument");
    return run_sim(&dec, 1, sp, FPLDPC_COLL_HOST, out, nullptr);
}

int fpldpc_ber_sim_multi(const fpldpc_decoder_t *decs, int32_t ndev, const fpldpc_sim_params *sp, int32_t collective,
                         fpldpc_sim_result *out, int32_t *collective_used) {
    return run_sim(decs, ndev, sp, collective, out, collective_used);
}

void fpldpc_testing_sim_inject(int32_t fail_rank, int64_t fail_round, int32_t abrupt, int32_t fail_comm_init) {
    g_inject.fail_rank = fail_rank;
    g_inject.fail_round = fail_round;
    g_inject.abrupt = abrupt != 0;
    g_inject.comm_init = fail_comm_init;
}

}  // extern "C"
