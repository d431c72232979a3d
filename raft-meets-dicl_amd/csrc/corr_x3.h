// corr_x3.h — internal interface of the fp32-accurate split-bf16 correlation GEMM (corr_pyramid_x3.hip).
#pragma once

#include "rmd_common.h"

namespace rmd {
namespace x3 {

// true when the x3 kernel handles this pyramid: fp32 storage, C <= 256, 32-bit store offsets
bool eligible(const rmd_pyramid_desc& d, int channels);
size_t workspace_bytes(const rmd_pyramid_desc& d);
int prepare(const float* fmap1, const float* fmap2, int channels, float scale, const rmd_pyramid_desc& d,
            void* workspace, hipStream_t st);
int pyramid(const rmd_pyramid_desc& d, void* pyramid, void* workspace, hipStream_t st);

}  // namespace x3
}  // namespace rmd
