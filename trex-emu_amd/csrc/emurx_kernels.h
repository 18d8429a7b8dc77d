// emurx_kernels.h — launcher of the rx parse / classify / queue kernels (emurx_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/emu_rx.h"
#include "emurx_tables.h"

// Frames per k_rx workgroup (one per lane) == tile of the queue compaction.
#define EMURX_TILE 256u
// Copies of the outcome histogram that workgroups add into (tile % SHARDS); the last k_q
// workgroup folds them into the caller's histogram and zeroes them again.
#define EMURX_HIST_SHARDS 64

// Launch control block (device memory, one per handle), {0} at creation; `done` counts
// finished k_q workgroups and is reset by the last one.
struct emurx_ctl {
    uint32_t done, rsv[3];
};

// Per-handle device scratch of a batch (sized for cfg.max_frames at emurx_open).
struct emurx_scratch {
    uint8_t* qtag;               // [max_frames] queue of each frame (k_rx -> k_q)
    uint32_t* tile_cnt;          // [max_tiles][16] queue counts per tile
    uint32_t* gsum;              // [max_tiles/64][16] queue totals per 64 tiles; zero between batches
    unsigned long long* hshard;  // [EMURX_HIST_SHARDS][2 * EMURX_HIST_BINS]; zero between batches
    emurx_ctl* ctl;
};

// Enqueue one batch on `st`: k_rx then k_q, no host synchronisation.  ev[0..2] (optional,
// all or none) are recorded before k_rx, between the kernels and after k_q.  Returns 0 / -1.
int emurx_launch_batch(const uint8_t* frames, const emurx_desc* desc, uint32_t n,
                       const emurx_dev_tables& T, bool classify, const emurx_dev_out& out,
                       const emurx_scratch& s, hipStream_t st, const hipEvent_t* ev);
