/*
 * drcvar_exchange.h — C ABI of the peer-push record exchange across the GPUs of one node.
 *
 * The QP hand-off (core/mpc_filter.py:116-151) takes every halfspace of the horizon, so a batch
 * sharded over the ranks of a node (core/halfspaces.py:225-246: units are independent) must be
 * reassembled on every rank.  The portable form is one RCCL all_gather_into_tensor of the records
 * (dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/sharding.py); this is the
 * MI355X-native one: every rank's halfspace launch writes each 64-B record straight into the
 * exchange region of EVERY rank (its own and, over xGMI, each peer's region mapped into this
 * process by IPC), so the exchange runs inside the kernel, and one small launch per step then
 * publishes this rank's generation, waits for every peer's, and copies the gathered records into
 * an ordinary device buffer.  No collective library, no host round trip; graph-capturable.
 *
 * Region of a rank (uncached device memory, drcvar_peer_alloc; doubles):
 *   [0, rows*8)              records of the steps of even generation (parity = generation & 1)
 *   [rows*8, 2*rows*8)       records of the steps of odd generation
 *   [2*rows*8, +64)          flags: uint64 per source rank, the last generation it finished
 * rows = n_ranks * per (per = units of one rank's block, the tail rank padded), record r at
 * r*8 in the [O*T, 8] order of drcvar_safe_halfspaces_f64 (DRCVAR_COL_*).
 *
 * Protocol per step g (= completed steps + 1): each rank's drcvar_safe_halfspaces_f64_peer writes
 * its rows of parity g & 1 into every region; drcvar_peer_signal_wait stores g into flag[rank] of
 * every region (system scope, after the launch before it has completed), waits until every
 * flag of its own region is >= g (bounded: spin_limit_us, then the error word is set and the
 * step's copy still happens), copies the parity buffer into `out` and advances the generation.
 * Double buffering makes it safe for a consumer on the same stream to read `out` between two
 * steps: a peer can only write parity g & 1 again after this rank has signalled step g + 1.
 */
#ifndef DRCVAR_EXCHANGE_H
#define DRCVAR_EXCHANGE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DRCVAR_MAX_PEERS 8
#define DRCVAR_PEER_HANDLE_BYTES 64 /* hipIpcMemHandle_t */

typedef struct drcvar_peer_set {
  double* region[DRCVAR_MAX_PEERS]; /* rank j's region, mapped in this process (region[rank] = own) */
  int64_t rows;                     /* records per parity buffer */
  unsigned long long* state;        /* this rank's device words: [0] generation, [1] launch counter
                                       (internal), [2] error (0 = ok; else bit j: rank j's flag never
                                       came, bit 63 set) — zero-initialised by the caller */
  int32_t n_ranks;                  /* 1..DRCVAR_MAX_PEERS */
  int32_t rank;
} drcvar_peer_set;

/* doubles of one rank's region for `rows` records per parity buffer */
int64_t drcvar_peer_region_doubles(int64_t rows);

/* Allocate a zeroed region (uncached device memory on the current device) and export its IPC
   handle (handle_out: DRCVAR_PEER_HANDLE_BYTES bytes, host). */
int drcvar_peer_alloc(int64_t doubles, double** region, void* handle_out);
int drcvar_peer_free(double* region);
/* Map a peer's region (its exported handle) into this process; access from the current device is
   enabled on the way (hipIpcMemLazyEnablePeerAccess). */
int drcvar_peer_open(const void* handle, double** region);
int drcvar_peer_close(double* region);
/* Whether `device` can access `peer_device`'s memory directly (1 for the same device). Host-only. */
int drcvar_peer_can_access(int32_t device, int32_t peer_device, int32_t* can_access);
/* The PCI bus id of `device` (host string, at most `len` bytes with the terminator), and the device
   of this process that has a given bus id (DRCVAR_ERR_UNSUPPORTED when this process does not see
   it): ranks name their GPUs to each other by bus id, since device indices differ between
   processes whose visible-device lists differ.  Host-only. */
int drcvar_peer_bus_id(int32_t device, char* bus_id, int32_t len);
int drcvar_peer_device_of(const char* bus_id, int32_t* device);

/* The step's publish + wait + copy (one launch on `stream`): out[rows * 8] doubles. */
int drcvar_peer_signal_wait(const drcvar_peer_set* peers, double* out, int64_t spin_limit_us,
                            void* stream);

/* The pull form of the step: every rank's halfspace launch wrote its rows into its OWN region only
   (drcvar_safe_halfspaces_f64_peer with the one-rank set {region = {own}, rows, state, n_ranks 1,
   rank 0}: no write round trip over xGMI per unit); this launch publishes and waits as
   drcvar_peer_signal_wait does and copies rank j's rows [j per, (j + 1) per) of the step's parity
   buffer from rank j's region.  rows must be n_ranks * per. */
int drcvar_peer_signal_wait_pull(const drcvar_peer_set* peers, double* out, int64_t spin_limit_us,
                                 void* stream);

/*
 * drcvar_safe_halfspaces_f64_v2 (include/drcvar_halfspace.h) in the peer-push form: unit u of the
 * launch (u = o * n_steps + t) is written to global row row_base + u of every rank's region in the
 * buffer of the step's parity, instead of to an `out` buffer.  Packed 16-B aligned samples only,
 * n_samples <= DRCVAR_MAX_SAMPLES, automatic geometry (DRCVAR_ERR_UNSUPPORTED otherwise).
 */
int drcvar_safe_halfspaces_f64_peer(const double* samples, int64_t n_obstacles, int64_t n_steps,
                                    int64_t n_samples, int64_t stride_obstacle, int64_t stride_step,
                                    int64_t stride_sample, const double* ego_ref_pos,
                                    int64_t ego_stride_step, double robot_radius,
                                    double obstacle_radius, double alpha, double delta,
                                    double epsilon, const drcvar_peer_set* peers, int64_t row_base,
                                    int32_t* status, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DRCVAR_EXCHANGE_H */
