// Homework kernel suite (hw1-hw4 capabilities) -- declarations.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
namespace cme {}
