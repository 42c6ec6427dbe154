// ingest.h -- host-side entry points of the file decoders (ingest.hip) that
// the drop-in's auto-ingest (host.cpp) uses beside the C-ABI ones.
#pragma once
#include <string>

#include "../../include/gskyhip.h"

namespace gsky {

// gskyhip_netcdf_info plus the dataset SRS for srs_cf = 0 and 1
// (gskyhip_netcdf_srs), from one read of the file.
int netcdf_info_srs(const char *path, gskyhip_raster_info *info, std::string *srs_no, std::string *srs_cf);

}  // namespace gsky
