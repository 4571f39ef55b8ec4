# make-compatible wrapper (reference Makefile:7-31 builds one ./a.out per
# program variant).  Here every variant is the same engine; the targets build
# it and install ./a.out as a thin wrapper that selects the matching style.
#
#   make            build the native module and CLI tools (gfx950)
#   make serial | game   ./a.out W H file  ->  bin/gol --style serial (CPU oracle engine is --engine ref)
#   make mpi | async | collective | openmp | cuda   (same engine, that variant's stdout lines)
#   make cmake      CMake build into build/cmake
#   make test       CPU test tier;  make test-gpu  MI355X tier
#   make bench      1-GPU benchmark JSON line
#   make selftest-asan / selftest-tsan   host runtime self test under ASan+UBSan / TSan
PYTHON ?= python3
JOBS ?= 8

.PHONY: all build game serial mpi async collective openmp cuda cmake test test-gpu bench selftest-asan selftest-tsan clean

all: build

build:
	$(PYTHON) game-of-life-in-parallel-mpi-openmp-cuda_amd/native_build.py

define AOUT
	@printf '#!/bin/sh\n# reference-compatible ./a.out (%s variant)\nexec "$$(dirname "$$0")/bin/gol" "$$@" --style %s $(2)\n' $(1) $(1) > a.out
	@chmod +x a.out
	@echo "./a.out -> bin/gol --style $(1) $(2)"
endef

serial: build
	$(call AOUT,serial,)
game: serial  # the reference's target name for the serial build (Makefile:12-13)
mpi: build
	$(call AOUT,mpi,)
async: build
	$(call AOUT,async,)
collective: build
	$(call AOUT,collective,)
openmp: build
	$(call AOUT,openmp,)
cuda: build
	$(call AOUT,cuda,--engine hip)

cmake:
	cmake -S . -B build/cmake -G Ninja && cmake --build build/cmake -j $(JOBS)

test: build
	$(PYTHON) -m pytest tests -x -q -m "not gpu"

test-gpu: build
	$(PYTHON) -m pytest tests -x -q -m gpu

bench: build
	$(PYTHON) bench.py

selftest-asan:
	$(PYTHON) game-of-life-in-parallel-mpi-openmp-cuda_amd/native_build.py --selftest address
	./bin/gol_selftest_address

selftest-tsan:
	$(PYTHON) game-of-life-in-parallel-mpi-openmp-cuda_amd/native_build.py --selftest thread
	TSAN_OPTIONS=halt_on_error=1 ./bin/gol_selftest_thread

clean:
	rm -rf build bin a.out game-of-life-in-parallel-mpi-openmp-cuda_amd/_gol.so
