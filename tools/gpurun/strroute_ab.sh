#!/bin/bash
# String[] route (dds_sum_all_dec): fused per-region length + copy fill (DDSHE_DEC_FUSE=1) against the
# length pass + copy pass (0), same box, after the codec tests with the fused fill on, the GPU suite and smoke.
export TMPDIR=/tmp
P="python3 -u tools/dec_route_probe.py --big --reps 9"
exec tools/gpurun/steps.sh \
  "300 codec_fused env DDSHE_DEC_FUSE=1 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_parity.py tests/test_gpu_moduli.py -x -q --timeout 250 --timeout-method thread" \
  "200 sr_Aa env DDSHE_DEC_FUSE=0 $P" "200 sr_Ba env DDSHE_DEC_FUSE=1 $P" \
  "200 sr_Ab env DDSHE_DEC_FUSE=0 $P" "200 sr_Bb env DDSHE_DEC_FUSE=1 $P" \
  "200 sr_B16 env DDSHE_DEC_FUSE=1 DDSHE_COPY_THREADS=16 $P" "200 sr_A16 env DDSHE_DEC_FUSE=0 DDSHE_COPY_THREADS=16 $P" \
  "700 tests python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "120 smoke python3 -c 'import __graft_entry__ as g; g.smoke()'"
