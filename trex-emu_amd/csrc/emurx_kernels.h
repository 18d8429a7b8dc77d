// emurx_kernels.h — launcher of the rx parse / classify / queue kernel (emurx_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/emu_rx.h"
#include "emurx_tables.h"

// Enqueue one batch on `st`: a single k_rx launch, no host synchronisation (capturable in a
// hipGraph).  ev[0..1] (optional) are recorded before and after it.  Returns 0 or -1.
int emurx_launch_batch(const uint8_t* frames, const emurx_desc* desc, uint32_t n,
                       const emurx_dev_tables& T, bool classify, const emurx_dev_out& out,
                       hipStream_t st, const hipEvent_t* ev);

// Enqueue the Namespace-partition packing of a classified batch (emurx_route.hip): three
// launches on `st`.  Scratch: tile_cnt [ceil(n / 256) * 16]; grp, grp_off [groups * 16] with
// groups = ceil(n / 16384) <= 1024 (n <= 16M); grp must be zero (the launches leave it zero).
int emurx_launch_route(const emurx_rec* rec, uint32_t n, uint32_t n_parts, uint32_t my_rank, uint32_t cap,
                       emurx_route_rec* send, uint32_t* send_count, uint32_t* tile_cnt, uint32_t* grp,
                       uint32_t* grp_off, hipStream_t st);
