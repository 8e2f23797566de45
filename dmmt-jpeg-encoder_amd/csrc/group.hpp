// group.hpp -- several GPUs behind one dmmt_ctx (dmmt_ctx_create_multi).
//
// The reference's only fan-out is a CPU thread pool: ThreadPool::new(n) at
// lib.rs:62, used by transform_on_threadpool (cosine_transform.rs:55-73) for the
// DCT.  Here the pool is one host thread per GPU, each driving one member context
// (an ordinary single-device dmmt_ctx), and the work it fans out is whole frames
// or MCU-row stripes of one image.  The group uses nothing but
// the public C ABI on its members; the single-device entry points of encoder.cpp
// forward to it when they are given a group.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/dmmt_jpeg.h"

namespace dmmt {

struct Group;

// creates one member context per id (repeats allowed: several contexts on one GPU)
int group_create(const int* device_ids, int n, Group** out);
void group_destroy(Group* g);
int group_size(const Group* g);
dmmt_ctx* group_member(Group* g, int i);

// frames round-robin over the members, one host thread each; outputs in input order
int group_encode_batch(Group* g, const dmmt_image* imgs, int n, const dmmt_options* opt, uint8_t** outs,
                       size_t* lens);
// one image as MCU-row stripes, one per member (n_stripes <= 0: every member)
int group_encode_striped(Group* g, const dmmt_image* img, const dmmt_options* opt, int n_stripes, uint8_t** out,
                         size_t* out_len);
// stripes already in the members' HBM (stripe i on member i), outputs in their HBM
int group_encode_striped_device(Group* g, const dmmt_stripe* stripes, int n, const dmmt_options* opt,
                                uint8_t* const* d_outs, const size_t* caps, uint64_t* lens);
// the same protocol over any contexts (workers: a Group's pool, or null = one after
// another on the calling thread); stripes in row order from MCU row 0
int stripes_on_contexts(dmmt_ctx* const* ctxs, void* workers, int n, const dmmt_stripe* stripes,
                        const dmmt_options* opt, uint8_t* const* d_outs, const size_t* caps, uint64_t* lens);
// device-resident frames, frames[i] on member i, enqueued without waiting
int group_encode_device(Group* g, const dmmt_device_frames* frames, int n, const dmmt_options* opt);
int group_synchronize(Group* g);
// every member checked on its worker thread (ctx_check_device + the group's staging buffers)
int group_check_devices(Group* g);
// encoder.cpp: the calling thread's device and every pooled buffer of c on c's GPU
int ctx_check_device(dmmt_ctx* c);
int ptr_check_device(const void* p, int device);
int group_set_lanes(Group* g, int n);
int group_set_profiling(Group* g, int enable);
int group_profile(Group* g, double* ms, int32_t* launches, int n_stages);

}  // namespace dmmt
