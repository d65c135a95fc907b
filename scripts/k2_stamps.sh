#!/bin/bash
timeout -k 10 120 python3 scripts/screen_stamps.py --lib nav-slam_amd/lib/variants/libnavgpu_stamps.so --pairs 1 2>&1 | tail -3
timeout -k 10 120 python3 scripts/screen_stamps.py --lib nav-slam_amd/lib/variants/libnavgpu_stamps.so --pairs 8 2>&1 | tail -3
