// capi.cpp — host-side parts of the C ABI: error state, version, pyramid geometry.
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "rmd.h"

namespace rmd {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

void clear_error() { g_err[0] = '\0'; }

static int level_chunk(int l) { return l <= 1 ? 8 : (l == 2 ? 4 : 2); }

}  // namespace rmd

extern "C" const char* rmd_last_error(void) { return rmd::g_err; }

extern "C" const char* rmd_version(void) { return "rmd 0.2 gfx950 abi 2"; }

extern "C" int rmd_abi_version(void) { return RMD_ABI_VERSION; }

// the Makefile's source fingerprint; the tagged string also lets rmd/_lib.py read it from the file
// without loading the library
#ifndef RMD_SRC_HASH
#define RMD_SRC_HASH "unknown"
#endif
static const char kSrcTag[] = "rmd-src-hash:" RMD_SRC_HASH;

extern "C" const char* rmd_source_hash(void) { return kSrcTag + 13; }

extern "C" int rmd_pyramid_describe_layout(int batch, int height, int width, int levels, int storage, int layout,
                                           rmd_pyramid_desc* d) {
    if (!d) {
        rmd::set_error("rmd_pyramid_describe: null desc");
        return RMD_ERR_ARG;
    }
    if (storage != RMD_F32 && storage != RMD_F16 && storage != RMD_S24) {
        rmd::set_error("rmd_pyramid_describe: storage must be RMD_F32, RMD_F16 or RMD_S24");
        return RMD_ERR_ARG;
    }
    if (layout != RMD_LAYOUT_ROWS && !(layout == RMD_LAYOUT_TILES && storage == RMD_F16)) {
        rmd::set_error("rmd_pyramid_describe: layout %d with storage %d (tiles need RMD_F16)", layout, storage);
        return RMD_ERR_ARG;
    }
    if (batch < 1 || height < 1 || width < 1 || levels < 1 || levels > RMD_MAX_LEVELS) {
        rmd::set_error("rmd_pyramid_describe: bad sizes (batch=%d height=%d width=%d levels=%d)", batch, height,
                       width, levels);
        return RMD_ERR_SHAPE;
    }
    std::memset(d, 0, sizeof(*d));
    d->batch = batch;
    d->height = height;
    d->width = width;
    d->levels = levels;
    d->storage = storage;
    d->layout = layout;
    const bool tiles = layout == RMD_LAYOUT_TILES;
    long long slots = (long long)height * width;
    if (tiles) {
        const long long qx = (width + 15) / 16;
        slots = (long long)(height / 2) * qx * 32 + ((height & 1) ? (long long)(width + 31) / 32 * 32 : 0);
    }
    if (slots > 0x7fffffffLL) {
        rmd::set_error("rmd_pyramid_describe: %lld query slots", slots);
        return RMD_ERR_SHAPE;
    }
    d->query_slots = (int)slots;
    long long off = 0;
    int h = height, w = width;
    for (int l = 0; l < levels; ++l) {
        if (h < 1 || w < 1) {
            // avg_pool2d of a 1-pixel map fails in the reference as well ("output size is too small")
            rmd::set_error("rmd_pyramid_describe: level %d of a %dx%d map is empty", l, height, width);
            return RMD_ERR_SHAPE;
        }
        const int th = tiles && l <= 1 ? 2 : 1;
        // S24 level 3: 1 x 4 chunks (12 bytes: one 4-aligned load) instead of 1 x 2
        const int tw = tiles ? (l <= 2 ? 4 : 2) : (storage == RMD_S24 && l == 3 ? 4 : rmd::level_chunk(l));
        d->level_h[l] = h;
        d->level_w[l] = w;
        d->tile_h[l] = th;
        d->tile_w[l] = tw;
        d->tiles_y[l] = (h + th - 1) / th;
        d->tiles_x[l] = (w + tw - 1) / tw;
        d->level_offset[l] = off;
        off += (long long)batch * d->tiles_y[l] * d->tiles_x[l] * slots * th * tw;
        h /= 2;
        w /= 2;
    }
    d->total_elements = off;
    rmd::clear_error();
    return RMD_OK;
}

extern "C" int rmd_pyramid_describe(int batch, int height, int width, int levels, int storage,
                                    rmd_pyramid_desc* d) {
    return rmd_pyramid_describe_layout(batch, height, width, levels, storage, RMD_LAYOUT_ROWS, d);
}
