// emurx_kernels.h — launcher of the rx parse / classify / compaction kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/emu_rx.h"
#include "emurx_tables.h"

// Frames per k_parse workgroup (one per lane) == tile of the queue compaction.
#define EMURX_TILE 256u

// Enqueue one batch on `st`.  tile_cnt / tile_off need ceil(n/EMURX_TILE)*16 + 16 words.
// ev0..ev2 (optional) bracket parse and compaction for timing.  Returns 0 or -1.
int emurx_launch_batch(const uint8_t* frames, const emurx_desc* desc, uint32_t n,
                       const emurx_dev_tables& T, bool classify, const emurx_dev_out& out,
                       emurx_rec* rec_scratch, uint8_t* qtag, uint32_t* tile_cnt,
                       uint32_t* tile_off, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1,
                       hipEvent_t ev2);
