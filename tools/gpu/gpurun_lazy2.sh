#!/bin/bash
timeout -k 10 400 python tools/ab.py base lazyv2 lazyv3 lazynochk base lazyv2 lazyv3 2>&1 | grep -v amdgpu.ids
