// transfer_dir.hpp -- TRANSFER_DIR of the reference's CLI programs
// (config/var-config.h.in: the project source directory, with "prm/" below it).
// Here: $TRANSFER_DIR if set, else <repo>/tests/golden/ located from the
// executable (<repo>/radiative-transfer_amd/bin/<exe>).
#pragma once

#include <unistd.h>

#include <cstdlib>
#include <string>

namespace rtamd {

inline std::string transfer_dir() {
  if (const char *e = std::getenv("TRANSFER_DIR")) return std::string(e);
  char buf[4096];
  const ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n > 0) {
    buf[n] = 0;
    std::string exe(buf);
    return exe.substr(0, exe.rfind('/')) + "/../../tests/golden/";
  }
  return "./";
}

}  // namespace rtamd
