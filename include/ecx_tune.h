/*
 * ecx_tune.h -- launch-shape knobs of libecx.so for diagnostics and tuning.
 * Not part of the reference's coding interface (include/ecx.h is the boundary);
 * results are bit-identical for every setting, only speed changes.
 *
 *   "items_per_block"  consecutive 4 KiB chunks one workgroup streams (default 8;
 *                      0 = one chunk per workgroup, the simple k_gf_apply form)
 *   "nontemporal"      1 = non-temporal (streaming) loads/stores in the streaming kernel
 */
#ifndef ECX_TUNE_H
#define ECX_TUNE_H
#ifdef __cplusplus
extern "C" {
#endif
int ecx_tune(const char *key, int value); /* 0, or ECX_E_ILLEGAL_ARGUMENT for an unknown key */
#ifdef __cplusplus
}
#endif
#endif
