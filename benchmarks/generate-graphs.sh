#!/usr/bin/env bash
# Reference used gnuplot (requests.p / memory.p); gnuplot is not in this image, matplotlib is.
cd "$(dirname "$0")"
python3 plots.py
