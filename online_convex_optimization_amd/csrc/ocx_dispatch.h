// ocx_dispatch.h — runtime layout (C, P, chain) → template instance of a launcher FN.
#pragma once

// (C, P) tree instances for every supported C; chain (exact mode, P > 1) instances for
// power-of-two C.
#define OCX_DISPATCH_P(FN, C, ...)                    \
    switch (L->P) {                                   \
        case 1: return FN<C, 1, false>(__VA_ARGS__);  \
        case 2: return FN<C, 2, false>(__VA_ARGS__);  \
        case 4: return FN<C, 4, false>(__VA_ARGS__);  \
        case 8: return FN<C, 8, false>(__VA_ARGS__);  \
        case 16: return FN<C, 16, false>(__VA_ARGS__); \
        case 32: return FN<C, 32, false>(__VA_ARGS__); \
        case 64: return FN<C, 64, false>(__VA_ARGS__); \
        default: return hipErrorInvalidValue;         \
    }

#define OCX_DISPATCH_CHAIN_P(FN, C, ...)             \
    switch (L->P) {                                  \
        case 2: return FN<C, 2, true>(__VA_ARGS__);  \
        case 4: return FN<C, 4, true>(__VA_ARGS__);  \
        case 8: return FN<C, 8, true>(__VA_ARGS__);  \
        case 16: return FN<C, 16, true>(__VA_ARGS__); \
        case 32: return FN<C, 32, true>(__VA_ARGS__); \
        case 64: return FN<C, 64, true>(__VA_ARGS__); \
        default: return hipErrorInvalidValue;        \
    }

#define OCX_DISPATCH(FN, ...)                                         \
    if (L->chain) {                                                   \
        switch (L->C) {                                               \
            case 2: OCX_DISPATCH_CHAIN_P(FN, 2, __VA_ARGS__)          \
            case 4: OCX_DISPATCH_CHAIN_P(FN, 4, __VA_ARGS__)          \
            case 8: OCX_DISPATCH_CHAIN_P(FN, 8, __VA_ARGS__)          \
            case 16: OCX_DISPATCH_CHAIN_P(FN, 16, __VA_ARGS__)        \
            case 32: OCX_DISPATCH_CHAIN_P(FN, 32, __VA_ARGS__)        \
            case 64: OCX_DISPATCH_CHAIN_P(FN, 64, __VA_ARGS__)        \
            default: return hipErrorInvalidValue;                     \
        }                                                             \
    }                                                                 \
    switch (L->C) {                                                   \
        case 2: OCX_DISPATCH_P(FN, 2, __VA_ARGS__)                    \
        case 4: OCX_DISPATCH_P(FN, 4, __VA_ARGS__)                    \
        case 6: OCX_DISPATCH_P(FN, 6, __VA_ARGS__)                    \
        case 8: OCX_DISPATCH_P(FN, 8, __VA_ARGS__)                    \
        case 12: OCX_DISPATCH_P(FN, 12, __VA_ARGS__)                  \
        case 16: OCX_DISPATCH_P(FN, 16, __VA_ARGS__)                  \
        case 24: OCX_DISPATCH_P(FN, 24, __VA_ARGS__)                  \
        case 32: OCX_DISPATCH_P(FN, 32, __VA_ARGS__)                  \
        case 48: OCX_DISPATCH_P(FN, 48, __VA_ARGS__)                  \
        case 64: OCX_DISPATCH_P(FN, 64, __VA_ARGS__)                  \
        default: return hipErrorInvalidValue;                         \
    }
