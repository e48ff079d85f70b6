#!/bin/bash
timeout -k 10 200 python tools/stamps.py 2>&1 | grep -v amdgpu.ids
