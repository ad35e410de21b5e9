# Images of this build. One repository, two tags, as upstream publishes
# rocm/k8s-device-plugin:<version> and :labeller-<version>:
#
#   $(IMAGE_REPO):$(VERSION)            device plugin   (Dockerfile, ubi-dp.Dockerfile: -ubi)
#   $(IMAGE_REPO):labeller-$(VERSION)   node labeller   (labeller.Dockerfile, ubi-labeller.Dockerfile: -ubi)
#
# VERSION is the chart's appVersion, so the manifests, the chart defaults and
# the built tags name the same image (tests/test_image_layout.py checks it).
# To deploy from your own registry: make images push IMAGE_REPO=<registry>/<name>
# and point the manifests / chart at it (docs/installation.md).
IMAGE_REPO ?= ghcr.io/mi355x/k8s-device-plugin
VERSION ?= $(shell sed -n 's/^appVersion: "\(.*\)"/\1/p' helm/amd-gpu/Chart.yaml)
GIT_DESCRIBE ?= $(shell git describe --always --long --dirty 2>/dev/null || echo $(VERSION))
DOCKER ?= docker
BUILD_ARGS = --build-arg GIT_DESCRIBE=$(GIT_DESCRIBE)

.PHONY: images push native test test-gpu sanitizers coverage fuzz bench

images:
	$(DOCKER) build $(BUILD_ARGS) -f Dockerfile -t $(IMAGE_REPO):$(VERSION) .
	$(DOCKER) build $(BUILD_ARGS) -f labeller.Dockerfile -t $(IMAGE_REPO):labeller-$(VERSION) .
	$(DOCKER) build $(BUILD_ARGS) -f ubi-dp.Dockerfile -t $(IMAGE_REPO):$(VERSION)-ubi .
	$(DOCKER) build $(BUILD_ARGS) -f ubi-labeller.Dockerfile -t $(IMAGE_REPO):labeller-$(VERSION)-ubi .

push:
	$(DOCKER) push $(IMAGE_REPO):$(VERSION)
	$(DOCKER) push $(IMAGE_REPO):labeller-$(VERSION)
	$(DOCKER) push $(IMAGE_REPO):$(VERSION)-ubi
	$(DOCKER) push $(IMAGE_REPO):labeller-$(VERSION)-ubi

native:
	python3 -m rocm_k8s_device_plugin_amd._build

test:
	python3 -m pytest tests -q -m "not gpu"

test-gpu:
	python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread

# ctest under ASan+UBSan and under TSan (host-only builds in build/native-<sanitizer>)
sanitizers:
	python3 -m rocm_k8s_device_plugin_amd._build --no-hip --sanitize address,undefined --ctest
	python3 -m rocm_k8s_device_plugin_amd._build --no-hip --sanitize thread --ctest

# gcov line coverage of the native host code by the CPU suite (docs/development.md)
coverage:
	python3 tools/native_coverage.py --json-out build/native_coverage.json

# libFuzzer over every native parser (clang), 60 s per target
fuzz:
	python3 tools/fuzz_native.py --seconds 60 --json build/fuzz_native.json

# the headline benchmark on this node (needs an MI355X)
bench:
	python3 bench.py --gpus 1 --steps 20 --warmup 3
