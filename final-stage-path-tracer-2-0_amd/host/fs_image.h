// fs_image.h — texture file loaders of the reference's material path.
//
//  LoadBitmap  restates bitmap.cpp:40-104 (24-bit BMP, rows as stored).
//  LoadEXR     restates the LoadEXR() entry point of the tinyexr header the
//              reference vendors (source/third_party/tiny_exr_loader.h:11179)
//              for scanline and one-level tiled files with NONE, RLE, ZIPS or
//              ZIP compression (zlib inflate) and HALF/FLOAT/UINT channels.
//              PIZ, which tinyexr also decodes, is reported as unsupported.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

namespace base {

// bitmap.cpp:40: returns false on failure; like the reference, a file that
// fails after the header has been read leaves output resized (zero texels)
// and width/height set.
bool LoadBitmap(const std::string& filename, std::vector<float>* output, uint32_t* width, uint32_t* height);

// tiny_exr_loader.h:11179: *out_rgba = malloc'd RGBA floats (free()), 0 on
// success, a negative tinyexr error code otherwise with *err set.
int LoadEXR(float** out_rgba, int* width, int* height, const char* filename, const char** err);

}  // namespace base
