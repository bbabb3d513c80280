#!/bin/bash
# round 5: sessions o then n in one call (the pool had no free box for n alone)
bash tools/sessions/gpu_r5o.sh && bash tools/sessions/gpu_r5n.sh
