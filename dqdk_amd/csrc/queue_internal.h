/*
 * queue_internal.h -- runtime-internal entry points of dqdk_gpu.hip used by
 * the other host translation units of libdqdk_gpu.so (not exported).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dqdk_gpu.h"

namespace dqdk {

// One frame-processor batch on the queue stream (async): n staged payloads
// of queue_events(q) * 16 bytes at d_stage and their datalens at d_len (both
// DEVICE, valid until the stream reaches the launch) through fp_decode,
// rx_count and the records-path histogram.  n <= the queue's max_batch.
int queue_launch_payloads(dqdk_gpu_queue_t* q, const uint8_t* d_stage, const uint32_t* d_len, uint32_t n);
int queue_device(const dqdk_gpu_queue_t* q);
// events a payload carries for the histogram (0: the mode keeps none)
uint32_t queue_events(const dqdk_gpu_queue_t* q);
// dqdk_gpu_last_error() of the calling thread; return err / -EIO
int set_error(int err, const char* what);
int set_hip_error(const char* what, hipError_t e);

}  // namespace dqdk
