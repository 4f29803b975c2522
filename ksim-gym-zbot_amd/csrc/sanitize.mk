# Host sanitizer build of the C ABI's host-only half (tests/test_sanitizers.py).
# g++ only, no GPU code: zb_host.cpp (model / config validation, team topology, defaults) linked
# with the mutation driver zb_host_selftest.cpp.
#   make -C ksim-gym-zbot_amd/csrc -f sanitize.mk
CXX ?= g++
SAN = -fsanitize=address,undefined -fsanitize=bounds -fno-sanitize-recover=all -fno-omit-frame-pointer
OBJDIR ?= build
$(OBJDIR)/zb_host_selftest: zb_host.cpp zb_host.h zb_host_selftest.cpp ../../include/zbot.h ../../include/zbot_model.h ../../include/zbot_layout.h
	@mkdir -p $(OBJDIR)
	$(CXX) -std=c++17 -O1 -g $(SAN) -Wall -I../../include -o $@ zb_host.cpp zb_host_selftest.cpp
