# LDS-DMA conv tile sweep (S2V_GLDS_TILE = conv.hip kGlds index), one process per tile
set -e
for t in ${T256:-0}; do S2V_GLDS_TILE=$t timeout -k 10 120 python tools/conv_micro.py --n 16 --h 256 --w 256 --cin 256 --cout 256 --prec f16x3 --glds --iters 10 2>&1 | grep "glds conv" | sed "s/^/T$t 256sq /"; done
for t in ${T400:-1 2}; do S2V_GLDS_TILE=$t timeout -k 10 120 python tools/conv_micro.py --n 16 --h 400 --w 400 --cin 256 --cout 128 --prec f16x3 --glds --iters 5 2>&1 | grep "glds conv" | sed "s/^/T$t 400-256 /"; done
for t in ${T400B:-1 2}; do S2V_GLDS_TILE=$t timeout -k 10 120 python tools/conv_micro.py --n 16 --h 400 --w 400 --cin 128 --cout 128 --prec f16x3 --glds --iters 5 2>&1 | grep "glds conv" | sed "s/^/T$t 400-128 /"; done
