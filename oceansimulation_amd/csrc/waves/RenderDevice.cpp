// RenderDevice.cpp — HIP-backed Vision::RenderDevice shim (see include/vision/RenderDevice.h).
#include "vision/RenderDevice.h"

#include <stdexcept>
#include <string>

namespace Vision
{

static void check(hipError_t e, const char* what)
{
  if (e != hipSuccess)
    throw std::runtime_error(std::string("Vision::RenderDevice: ") + what + ": " + hipGetErrorString(e));
}

RenderDevice::RenderDevice(hipStream_t s) : stream(s) {}

RenderDevice::~RenderDevice()
{
  for (auto& kv : textures)
    if (kv.second.owned && kv.second.ptr)
      (void)hipFree(kv.second.ptr);
}

const RenderDevice::Texture& RenderDevice::Get(ID id) const
{
  auto it = textures.find(id);
  if (it == textures.end())
    throw std::runtime_error("Vision::RenderDevice: unknown texture ID " + std::to_string(id));
  return it->second;
}

ID RenderDevice::CreateTexture2D(const Texture2DDesc& desc)
{
  Texture t;
  t.width = desc.Width;
  t.height = desc.Height;
  t.type = desc.PixelType;
  t.owned = true;
  const std::size_t bytes = t.width * t.height * BytesPerTexel(t.type);
  check(hipMalloc(&t.ptr, bytes), "hipMalloc");
  if (desc.Data)
    check(hipMemcpy(t.ptr, desc.Data, bytes, hipMemcpyHostToDevice), "hipMemcpy");
  else
    check(hipMemsetAsync(t.ptr, 0, bytes, stream), "hipMemsetAsync");
  ID id = nextID++;
  textures[id] = t;
  return id;
}

ID RenderDevice::RegisterTexture2D(void* ptr, std::size_t w, std::size_t h, PixelType type)
{
  Texture t;
  t.ptr = ptr;
  t.width = w;
  t.height = h;
  t.type = type;
  t.owned = false;
  ID id = nextID++;
  textures[id] = t;
  return id;
}

void RenderDevice::DestroyTexture2D(ID id)
{
  auto it = textures.find(id);
  if (it == textures.end())
    return;
  if (it->second.owned && it->second.ptr)
  {
    check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    check(hipFree(it->second.ptr), "hipFree");
  }
  textures.erase(it);
}

void RenderDevice::SetTexture2DDataRaw(ID id, const void* data)
{
  const Texture& t = Get(id);
  check(hipMemcpyAsync(t.ptr, data, t.width * t.height * BytesPerTexel(t.type), hipMemcpyHostToDevice, stream),
        "hipMemcpyAsync");
  check(hipStreamSynchronize(stream), "hipStreamSynchronize");
}

void RenderDevice::GetTexture2DDataRaw(ID id, void* out)
{
  const Texture& t = Get(id);
  check(hipMemcpyAsync(out, t.ptr, t.width * t.height * BytesPerTexel(t.type), hipMemcpyDeviceToHost, stream),
        "hipMemcpyAsync");
  check(hipStreamSynchronize(stream), "hipStreamSynchronize");
}

void* RenderDevice::GetTexturePointer(ID id) const { return Get(id).ptr; }
std::size_t RenderDevice::GetTextureWidth(ID id) const { return Get(id).width; }
std::size_t RenderDevice::GetTextureHeight(ID id) const { return Get(id).height; }
PixelType RenderDevice::GetTexturePixelType(ID id) const { return Get(id).type; }

void RenderDevice::SubmitCommandBuffer() { check(hipStreamSynchronize(stream), "hipStreamSynchronize"); }

}  // namespace Vision
