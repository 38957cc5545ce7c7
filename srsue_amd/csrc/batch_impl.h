// batch_impl.h -- the opaque mi_dl_batch_t of include/mi_dl.h (shared by batch.cpp and ctrl.cpp).
#pragma once
#include <vector>

#include "engine.h"

struct mi_dl_batch {
  mi::Engine eng;
  std::vector<mi_dl_sf_cfg_t> cfgs;
};
