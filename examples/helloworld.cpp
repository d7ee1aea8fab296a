// helloworld.cpp -- minimal use of the drop-in API, mirroring the reference's
// helloworld.cpp (32 random keys, sortKeys over bits [0,32), print).  Unlike
// the reference (helloworld.cpp:52-58) it synchronises the stream before the
// read-back.
#include <thrs/tinyhipradixsort.hpp>

#include <cstdio>
#include <cstdlib>
#include <memory>
#include <vector>

int main() {
  hipStream_t stream = nullptr;
  thrs::check(thrs_stream_create(&stream));
  {
    std::vector<std::string> extraArgs;
    thrs::RadixSort::Config config;
    config.configureWithKey<uint32_t>();
    thrs::RadixSort radixsort(extraArgs, config);

    std::vector<uint32_t> inputs(32);
    for (auto& x : inputs) x = rand();
    uint32_t numberOfInputs = inputs.size();
    std::unique_ptr<thrs::Buffer> inputKeyBuffer(new thrs::Buffer(sizeof(uint32_t) * inputs.size()));
    thrs::check(thrs_memcpy_htod_async(inputKeyBuffer->data(), inputs.data(), sizeof(uint32_t) * inputs.size(), stream));

    thrs::Buffer tmpBuffer(radixsort.getTemporaryBufferBytes(numberOfInputs).getTemporaryBufferBytesForSortKeys());
    radixsort.sortKeys(inputKeyBuffer->data(), numberOfInputs, tmpBuffer.data(), 0, 32, stream);

    thrs::check(thrs_stream_synchronize(stream));
    std::vector<uint32_t> outputs(inputs.size());
    thrs::check(thrs_memcpy_dtoh(outputs.data(), inputKeyBuffer->data(), sizeof(uint32_t) * outputs.size()));
    for (uint32_t i = 0; i < numberOfInputs; i++) std::printf("%u\n", outputs[i]);
  }
  thrs_stream_destroy(stream);
  return 0;
}
