// pt_dev.h — the device-level API behind the exported C ABI: one part of a libpt context, i.e. the
// effects, textures, render targets and draws of one HIP stream on one gfx950 device
// (pt_capi.cpp). The exported pt_* functions (include/pt.h, pt_group.cpp) own one Dev per part of
// a context and forward each call to every part; the signatures mirror pt.h's one for one.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/pt.h"

struct Dev;
struct DevTex;
struct DevFx;

Dev* dev_ctx_create(int device, int* err);
void dev_ctx_destroy(Dev* c);
const char* dev_last_error(Dev* c);
int dev_sync(Dev* c);
int dev_canvas_resize(Dev* c, int width, int height);
int dev_canvas_wrap(Dev* c, int width, int height, void* device_ptr);
int dev_set_output_partition(Dev* c, int enable);
DevFx* dev_effect_create(Dev* c, const char* src, const char* const* un, int nu, const char* const* sn, int ns, int* err);
DevFx* dev_effect_create_program(Dev* c, int prog, const char* const* un, int nu, const char* const* sn, int ns, int* err);
void dev_effect_destroy(DevFx* fx);
int dev_effect_program(const DevFx* fx);
int dev_set_float(DevFx* fx, const char* name, const float* v, int n);
int dev_set_int(DevFx* fx, const char* name, int v);
int dev_set_texture(DevFx* fx, const char* name, DevTex* t);
DevTex* dev_texture_create_rgba32f(Dev* c, int w, int h, const float* data, int sampling, int invert_y, int* err);
DevTex* dev_texture_create_rgba8(Dev* c, int w, int h, const uint8_t* data, int sampling, int invert_y, int* err);
DevTex* dev_render_target_create(Dev* c, int w, int h, int* err);
DevTex* dev_render_target_wrap(Dev* c, int w, int h, void* dptr, int* err);
int dev_render_target_resize(DevTex* t, int w, int h);
int dev_texture_size(const DevTex* t, int* w, int* h);
void dev_texture_destroy(DevTex* t);
int dev_render(DevFx* fx, DevTex* target);
int dev_read_pixels(Dev* c, const DevTex* t, void* dst, size_t bytes);
int dev_write_pixels(Dev* c, DevTex* t, const void* src, size_t bytes);
int dev_set_stream(Dev* c, void* stream);
int dev_set_backend(Dev* c, int backend);
int dev_set_bvh_layout(Dev* c, int layout);
int dev_bvh_layout_used(Dev* c);
int dev_set_row_partition(Dev* c, int num_parts, int part);
void* dev_texture_device_ptr(DevTex* t);
int dev_last_render_ms(Dev* c, int prog, float* ms);
int dev_timing_begin(Dev* c);
int dev_timing_end(Dev* c, int prog, double* total_ms, int* launches);
int dev_set_counting(Dev* c, int enable);
int dev_read_counters(Dev* c, uint64_t out[PT_NUM_COUNTERS]);
int dev_reset_counters(Dev* c);
int dev_timing_latency(Dev* c, int prog, float* ms, int cap, int* n);
int dev_queue_stats(Dev* c, uint32_t out[16]);
int dev_math_exhaustive(Dev* c, int op, uint64_t* mismatches);
int dev_math_probe(Dev* c, int op, const float* x, const float* y, float* out, int n);

// for the multi-part layer (pt_group.cpp): the part's device and stream, its canvas, and running a
// deferred screenCopy now (without a host sync) before another part reads this part's targets
int dev_device(const Dev* c);
hipStream_t dev_stream(const Dev* c);
void* dev_canvas_ptr(Dev* c);
int dev_flush(Dev* c);
