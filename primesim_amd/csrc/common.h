// common.h — host-side helpers shared by the C-ABI translation units.
#pragma once

#include <string>

namespace pu {

// Records a message for pu_last_error() and returns `code`.
int set_error(int code, const std::string& msg);

}  // namespace pu
