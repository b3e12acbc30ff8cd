// soundmath/delaybank.h -- Delaybank<T,N> lives with Delay<T> (delay.h).
#pragma once
#include "delay.h"
