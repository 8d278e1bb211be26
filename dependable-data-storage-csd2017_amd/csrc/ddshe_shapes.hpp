// Instantiated lane-group shapes and the runtime S -> template dispatch used by the launchers.
#pragma once
#include "ddshe_launch.hpp"

namespace ddshe {

// Instantiated shapes (S limbs of W bits on TPI lanes); a modulus uses the first that holds
// bits+2 bits. Keep in sync with kShapes below.
#define DDSHE_DISPATCH(S_, TPI_, W_, ...)            \
  case S_: {                                         \
    constexpr int S = S_, TPI = TPI_, W = W_;        \
    __VA_ARGS__;                                     \
  } break;

#define DDSHE_SWITCH(S_RT, ...)                      \
  switch (S_RT) {                                    \
    DDSHE_DISPATCH(40, 2, 28, __VA_ARGS__)           \
    DDSHE_DISPATCH(74, 2, 28, __VA_ARGS__)           \
    DDSHE_DISPATCH(76, 2, 28, __VA_ARGS__)           \
    DDSHE_DISPATCH(112, 4, 28, __VA_ARGS__)          \
    DDSHE_DISPATCH(148, 4, 28, __VA_ARGS__)          \
    DDSHE_DISPATCH(232, 8, 27, __VA_ARGS__)          \
    DDSHE_DISPATCH(320, 16, 27, __VA_ARGS__)         \
    DDSHE_DISPATCH(640, 32, 27, __VA_ARGS__)         \
    default: return hipErrorInvalidValue;            \
  }

// 320 x 27 bits: an 8192-bit modulus (n^2 of a 4096-bit Paillier key, QP-capable); 640 x 27: up to
// 17278 bits (the JDK's largest RSA modulus, 16384 bits, for MultAll's pubkey). Wide shapes keep
// L = S/TPI = 20 limbs per lane (register budget) and serve as their own tail shapes.
// {76, 2, 28} is the 2048-bit alternative to {74, 2, 28} (4-limb blocks, room for the QP modulus);
// pick_shape uses 76 unless DDSHE_RSA76=0
inline constexpr Shape kShapes[] = {{40, 2, 28},  {74, 2, 28},   {76, 2, 28},   {112, 4, 28},
                                    {148, 4, 28}, {232, 8, 27},  {320, 16, 27}, {640, 32, 27}};
// latency-oriented shapes for the reduction tree / finalize: 16 lanes per bignum (32 for the widest)
inline constexpr Shape kTail[] = {{48, 16, 28},  {80, 16, 28},  {80, 16, 28},   {112, 16, 28},
                                  {160, 16, 28}, {240, 16, 27}, {320, 16, 27}, {640, 32, 27}};

#define DDSHE_TAIL_SWITCH(S_RT, ...)                 \
  switch (S_RT) {                                    \
    DDSHE_DISPATCH(48, 16, 28, __VA_ARGS__)          \
    DDSHE_DISPATCH(80, 16, 28, __VA_ARGS__)          \
    DDSHE_DISPATCH(112, 16, 28, __VA_ARGS__)         \
    DDSHE_DISPATCH(160, 16, 28, __VA_ARGS__)         \
    DDSHE_DISPATCH(240, 16, 27, __VA_ARGS__)         \
    DDSHE_DISPATCH(320, 16, 27, __VA_ARGS__)         \
    DDSHE_DISPATCH(640, 32, 27, __VA_ARGS__)         \
    default: return hipErrorInvalidValue;            \
  }

static inline unsigned grid_for(size_t threads) { return (unsigned)((threads + 255) / 256); }

}  // namespace ddshe
