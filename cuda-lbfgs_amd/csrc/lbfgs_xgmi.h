// lbfgs_xgmi.h — internal interface of the xGMI peer exchange (lbfgs_xgmi.hip).
//
// Sharded runs (one process per GPU) need, after every reduction, the 8 group partials of a
// result slot on every rank. Each rank owns groups [g_lo, g_hi) of the slot.
// This module moves them GPU to GPU without a collective library: every rank owns a small
// mailbox in uncached device memory, exported by IPC handle; a one-workgroup kernel stores the
// rank's own group values straight into each peer's mailbox over xGMI and then polls its own
// mailbox until every peer's values of this exchange have arrived.
//
// Wire format (the LL idea: data and flag in one 8-byte store, so no fences and no separate
// flag): each double travels as two 64-bit words (epoch << 32 | 32 data bits). The epoch is
// a per-context counter that every rank advances identically (the sharded solver issues the
// same exchanges in the same order on every rank); the mailbox is double-buffered by epoch
// parity, so a rank that has finished exchange e and already writes e + 1 never overwrites
// values a slower peer still has to read for e.
#ifndef LBFGS_XGMI_H
#define LBFGS_XGMI_H
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#define LBK_PEER_HANDLE_BYTES 64

struct lbk_xgmi;

// allocate the mailbox on `device` (current device must be `device`); positions = the most
// doubles one slot holds (LBK_GROUPS * widest stride)
int lbk_xgmi_create(lbk_xgmi** out, int device, int rank, int world, int positions, char* err, size_t cap);
void lbk_xgmi_destroy(lbk_xgmi* x);
// this rank's mailbox handle (LBK_PEER_HANDLE_BYTES)
int lbk_xgmi_handle(const lbk_xgmi* x, void* out);
// map every peer's mailbox (handles: world entries in rank order) and run a self-test of
// `rounds` exchanges on `stream` (values checked bit for bit); 0 on success
int lbk_xgmi_connect(lbk_xgmi* x, const void* handles, hipStream_t stream, char* err, size_t cap);
int lbk_xgmi_connected(const lbk_xgmi* x);
// slot = [LBK_GROUPS][ks] doubles in device memory; this rank's groups [g_lo, g_hi) are final;
// afterwards (in stream order) every group is. host_mirror (a device-mapped host pointer to
// the same layout, or NULL) receives all groups as well, so the host reads the slot with no copy
int lbk_xgmi_exchange(lbk_xgmi* x, hipStream_t stream, double* slot, int ks, int g_lo, int g_hi,
                      double* host_mirror);
// raw 64-bit words of the same layout (integer sums such as the trace checksums)
int lbk_xgmi_exchange_u64(lbk_xgmi* x, hipStream_t stream, uint64_t* slot, int ks, int g_lo, int g_hi);
// nonzero once an exchange timed out waiting for a peer (the slot then holds NaN)
int lbk_xgmi_failed(const lbk_xgmi* x);

// ---- the exchange folded into the passes ----------------------------------------
// A pass kernel pushes its own group values (and a rank-edge value) into the peers' mailboxes
// itself, in the wire format above, and the consuming pass's prologue polls its own mailbox: no
// exchange kernel and no extra kernel boundary between the two passes. What the kernels need:
struct lbk_xgmi_fold {
    unsigned long long* const* peers;  // device array [world]: every rank's mailbox as mapped here
    const unsigned long long* own;     // this rank's mailbox
    unsigned* err;                     // pinned: set by a poll that timed out
    unsigned* errd;                    // the same flag in device memory, read by waiting polls
    unsigned long long timeout;        // wall-clock ticks
    int positions;                     // doubles per parity (the mailbox's [2][positions][2] layout)
    int rank, world;
    int shared_device;  // some peer's mailbox lives on this rank's own GPU (ranks sharing a device)
};
int lbk_xgmi_fold_info(const lbk_xgmi* x, lbk_xgmi_fold* out);  // -5 before a successful connect
// the epoch of the next exchange (the counter the exchange kernel advances, shared)
unsigned lbk_xgmi_next_epoch(lbk_xgmi* x);
// the fallback when no pass consumes a folded exchange: wait for the peers' pushes of `epoch`
// (component 0 of every other rank's groups, and with `edges` their rank-edge components 1 / 2)
// and write them into the slot
int lbk_xgmi_collect(lbk_xgmi* x, hipStream_t stream, double* slot, int ks, int g_lo, int g_hi, unsigned epoch,
                     int edges);

#endif
