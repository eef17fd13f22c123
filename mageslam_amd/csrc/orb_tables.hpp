// orb_tables.hpp — pre-rotated BRIEF sampling tables (30 rotations x 256 tests x (x0,y0,x1,y1)),
// data of OpenCVModified.cpp:74-138 (bit_pattern_31_rotated / bit_pattern_15_rotated), embedded
// from mageslam_amd/data/*.bin by tables.cpp.
#pragma once
#include <cstdint>

extern "C" const int8_t mage_bit_pattern_15_rotated[30 * 1024];
extern "C" const int8_t mage_bit_pattern_31_rotated[30 * 1024];
