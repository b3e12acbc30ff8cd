// soundmath/staticSTFT.h -- StaticSTFT lives with Fourier (fourier.h), as in the reference's
// pair of headers (src/staticSTFT.h).
#pragma once
#include "fourier.h"
