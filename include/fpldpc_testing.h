/* fpldpc_testing.h -- test-only entry points of libfpldpc.so.
 *
 * NOT part of the drop-in interface (include/fpldpc.h) and with no reference counterpart: fault
 * injection for the tests of the multi-decoder simulation (fpldpc_ber_sim_multi), set explicitly by
 * a test program through this call.  Nothing in the library reads them from the environment, so a
 * production run is never affected unless it calls this function. */
#ifndef FPLDPC_TESTING_H
#define FPLDPC_TESTING_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Process-wide, for the next fpldpc_ber_sim_multi calls until reset (fail_rank = -1, fail_comm_init = 0):
 *   fail_rank >= 0   rank `fail_rank` fails in round `fail_round` as a device error would -- reported
 *                    through the round's all-gather, or with abrupt != 0 by leaving the loop before it
 *                    (every other rank must stop either way, not hang);
 *   fail_comm_init   1: the RCCL communicator set-up fails as if ncclCommInitAll had returned an
 *                    error (FPLDPC_COLL_RCCL: the call fails; FPLDPC_COLL_AUTO: host exchange, reported
 *                    in collective_used); 2: the same, and FPLDPC_COLL_AUTO with a single decoder
 *                    attempts RCCL too (it would not), so the AUTO fallback runs on a one-GPU box. */
void fpldpc_testing_sim_inject(int32_t fail_rank, int64_t fail_round, int32_t abrupt, int32_t fail_comm_init);

#ifdef __cplusplus
}
#endif
#endif /* FPLDPC_TESTING_H */
