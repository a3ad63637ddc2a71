// all_kernels.h — one translation unit with every production kernel and launcher plus the
// microbenchmark-only variants (ab_kernels.h), so a microbenchmark can time any of them directly.
#pragma once

#include "../../oceansimulation_amd/csrc/ocean_kernels.hip"
#include "../../oceansimulation_amd/csrc/launch_half.hip"
#include "../../oceansimulation_amd/csrc/launch_slab.hip"
#include "../../oceansimulation_amd/csrc/launch_fft.hip"
#include "k_rows_xp.h"
#include "../../oceansimulation_amd/csrc/device/k_rows_hp.h"
#include "ab_kernels.h"
#include "k_cols_small.h"
