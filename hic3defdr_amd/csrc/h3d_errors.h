// Thread-local error text shared by the translation units of libh3d.so
// (h3d_last_error() returns it).
#pragma once

namespace h3derr {

// formats the message, stores it for h3d_last_error(), returns `code`
int fail(int code, const char* fmt, ...);
const char* last();

}  // namespace h3derr
