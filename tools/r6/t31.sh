#!/bin/bash
# round 6 final: the multi-rank bench rehearsed on one GPU (gloo, ranks sharing cuda:0): N = 2 at 1920x1080,
# N = 4 at 960x540 (4 ranks' frame slots share one GPU's memory here): weak and strong scaling images
# bit-identical to one rank's
export TMPDIR=/tmp
bash tools/gpu_task.sh rehearse r6final_rehearse2 2 && bash tools/gpu_task.sh rehearse r6final_rehearse4 4 960 540
